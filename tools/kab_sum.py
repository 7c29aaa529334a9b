"""mean gradient / update ms per variant of a tools/gpu_kab.sh log: python tools/kab_sum.py <log>"""
import collections, json, sys
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    if line.startswith("{"):
        j = json.loads(line)
        d[j["tag"]].append((j["grad_ms"], j["update_ms"]))
for k, v in d.items():
    g = [x[0] for x in v]
    print(f"{k:12s} grad {' '.join(f'{x:.4f}' for x in g)}  mean {sum(g) / len(g):.4f}  update mean {sum(x[1] for x in v) / len(v):.4f}")

"""Condense a tools/profile_round.sh run into committed files under profiles/:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary of the bench command
  profiles/<tag>_summary.md         per-kernel table (timed-trajectory launches) + PMC traffic
  profiles/<tag>_pmc.json           HBM bytes per gradient launch (gfx950-corrected)
usage: python tools/summarize_profile.py <tag> <out_dir>"""
import csv, glob, json, os, shutil, statistics, sys

tag, out = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(root, "profiles")
os.makedirs(prof, exist_ok=True)


def find(sub, pattern):
    hits = glob.glob(os.path.join(out, sub, "**", pattern), recursive=True)
    return hits[0] if hits else None


stats = find("trace", "*kernel_stats.csv")
shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
trace = list(csv.DictReader(open(find("trace", "*kernel_trace.csv"))))
bench = json.loads(open(os.path.join(out, "bench_trace.json")).read().strip().splitlines()[-1])

# the timed trajectory: bench.py runs the network check's two trajectories (when the line
# carries network_check: an untimed one, then the timed one), the warmup trajectory, then the back-to-back measurement
# session (a 2-step leapfrog session), then the timed trajectory; each starts with
# one k_step_sizes launch (traj_prepare)
trace.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(trace) if "k_step_sizes" in r["Kernel_Name"]]
sampler = bench.get("sampler") or ("network" if "network-joint" in bench["config"]["workload"] else "branch")
# trajectories before the timed one: the network check, the warmup, and (branch sampler) the
# back-to-back session
t_ix = (2 if bench.get("network_check") else 0) + (1 if bench.get("warmup") else 0) + (1 if sampler == "branch" else 0) \
    + (1 if sampler == "network" else 0)   # the network line's settling trajectory
timed = trace[starts[t_ix]:starts[t_ix + 1] if len(starts) > t_ix + 1 else len(trace)] if len(starts) > t_ix else []
tgrad = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in timed if "k_fused_grad" in r["Kernel_Name"]]
tupd = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in timed if "k_update" in r["Kernel_Name"]]
tspan = ((int(timed[-1]["End_Timestamp"]) - int(timed[0]["Start_Timestamp"])) / 1e6) if timed else 0.0

# launches of the gradient kernel over the full branch set (grid = items x 576 threads)
grad = [r for r in trace if "k_fused_grad" in r["Kernel_Name"]]
big = max(int(r["Grid_Size_X"]) for r in grad)
full = [r for r in grad if int(r["Grid_Size_X"]) == big]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in full]
upd_rows = [x for x in trace if "k_update" in x["Kernel_Name"]]
upd = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in upd_rows
       if int(r["Grid_Size_X"]) == max(int(x["Grid_Size_X"]) for x in upd_rows)] if upd_rows else []
# every kernel of the timed trajectory (e.g. the network sampler's forward-only launch)
per_kernel = {}
for r in timed:
    k = r["Kernel_Name"].split("(")[0]
    per_kernel.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)


def pmc_bytes(sub, counter, pick=statistics.median, kernel="k_fused_grad"):
    f = find(sub, "*counter_collection.csv")
    rows = list(csv.DictReader(open(f)))
    per = {}
    for r in rows:
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per.setdefault(key, [int(r["Grid_Size"]) if "Grid_Size" in r else 0, 0.0])
            per[key][1] += float(r["Counter_Value"])
    if not per:
        return None
    vals = [v for g, v in per.values()]
    gmax = max(g for g, v in per.values())
    vals = [v for g, v in per.values() if g == gmax]
    return pick(vals) * 1024.0  # rocprofv3 reports KB


fetch = pmc_bytes("fetch", "FETCH_SIZE") * 2.0   # gfx950: FETCH_SIZE counts 1/2 of wide streaming reads
# the steady-state leapfrog launch writes only the partial slabs; the first and
# last launch of a trajectory also write the n predictions per branch (4 n B)
write = pmc_bytes("write", "WRITE_SIZE", min)
write_pred = pmc_bytes("write", "WRITE_SIZE", max)
# the network sampler's forward-only launch (k_forward_gsum, the group-sum forward of every step but the
# last; k_forward_fx / k_forward_fi), when the command ran one
fwd_fetch = None
for fk in ("k_forward_gsum", "k_forward_fx", "k_forward_fi"):
    fb = pmc_bytes("fetch", "FETCH_SIZE", kernel=fk)
    if fb is not None:
        fwd_fetch = (fk, fb * 2.0)
        break
pmc = {"kernel": full[0]["Kernel_Name"], "config": bench["config"]["workload"],
       "timed_trajectory_grad_ms_mean": statistics.mean(tgrad) if tgrad else None,
       "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
       "traffic_bytes_per_launch": fetch + write, "write_bytes_trajectory_end_launch": write_pred,
       "alg_bytes_per_launch": bench["roofline"]["alg_bytes_per_launch"],
       "note": "FETCH_SIZE x 2 (gfx950 wide-read correction, MI355X_MICROARCH.md HBM), WRITE_SIZE as reported; "
               "fetch: median over the full-branch-set launches of a separate --pmc pass; write: the steady-state "
               "leapfrog launch (min; the trajectory's first and last launch also write predictions)"}
mf = find("mfma", "*counter_collection.csv")
if mf:  # MFMA utilisation pass: per-counter medians over the full-branch-set gradient launches
    per = {}
    for r in csv.DictReader(open(mf)):
        if "k_fused_grad" not in r["Kernel_Name"]:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        d = per.setdefault(key, {"grid": int(r.get("Grid_Size", 0) or 0)})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    gmax = max(d["grid"] for d in per.values())
    sel = [d for d in per.values() if d["grid"] == gmax]
    names = sorted({k for d in sel for k in d if k != "grid"})
    med = {k: statistics.median(d.get(k, 0.0) for d in sel) for k in names}
    cycles = med.get("GRBM_GUI_ACTIVE", 0.0) / 8.0   # rocprofv3 sums GRBM over the 8 XCDs
    busy = med.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    pmc["mfma"] = {"counters_median_per_launch": med,
                   "kernel_cycles": cycles,
                   "mfma_busy_per_simd_cycle": busy / (cycles * 1024) if cycles else None,
                   "mfma_busy_per_cu_cycle": busy / (cycles * 256) if cycles else None,
                   "note": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x SIMDs or CUs): the matrix pipes' busy "
                           "fraction over the launch; MOPS counters are the MFMA operation counts per launch"}
json.dump(pmc, open(os.path.join(prof, f"{tag}_pmc.json"), "w"), indent=1)

with open(os.path.join(prof, f"{tag}_summary.md"), "w") as f:
    f.write(f"# Profile {tag}: `rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline "
            f"{' '.join(sys.argv[3:])}`\n\n")
    f.write(f"workload: {bench['config']['workload']}\n\n")
    f.write(f"bench line under the profiler: value {bench['value']:.2f} {bench['unit']}, "
            f"ms_per_step {bench['ms_per_step']:.3f}\n\n")
    f.write("| kernel | launches (full branch set) | mean ms | median ms | min ms |\n|---|---|---|---|---|\n")
    f.write(f"| {full[0]['Kernel_Name']} | {len(dur)} | {statistics.mean(dur):.3f} | "
            f"{statistics.median(dur):.3f} | {min(dur):.3f} |\n")
    if upd:
        f.write(f"| k_update (full set) | {len(upd)} | {statistics.mean(upd):.3f} | {statistics.median(upd):.3f} | "
                f"{min(upd):.3f} |\n\n")
    else:
        f.write("\n(no separate update launches: the update runs in the gradient launch's tail)\n\n")
    if tgrad:
        f.write(f"**Timed trajectory** ({len(tgrad)} gradient launches, {len(tupd)} update launches, "
                f"span {tspan:.3f} ms for {bench['steps']} steps = {tspan / bench['steps']:.4f} ms per step): "
                f"gradient launch mean {statistics.mean(tgrad):.4f} ms (median {statistics.median(tgrad):.4f}), "
                f"update mean {statistics.mean(tupd) if tupd else 0.0:.4f} ms; "
                f"algorithmic bytes / mean gradient launch = "
                f"{pmc['alg_bytes_per_launch'] / (statistics.mean(tgrad) * 1e-3) / 1e9:.0f} GB/s = "
                f"{pmc['alg_bytes_per_launch'] / (statistics.mean(tgrad) * 1e-3) / 8e12:.3f} of 8 TB/s\n\n")
    if per_kernel:
        f.write("Every kernel of the timed trajectory:\n\n| kernel | launches | mean ms | total ms |\n|---|---|---|---|\n")
        for k, v in sorted(per_kernel.items(), key=lambda kv: -sum(kv[1])):
            f.write(f"| {k} | {len(v)} | {statistics.mean(v):.4f} | {sum(v):.3f} |\n")
        f.write("\n")
    f.write(f"bench.py's own HIP-event timing of the gradient launch: {bench['roofline']['kernel_ms']:.4f} ms "
            f"({bench['roofline'].get('kernel_ms_source', '')}); back-to-back "
            f"{bench['roofline'].get('kernel_ms_back_to_back') or float('nan'):.4f} ms\n\n")
    f.write(f"HBM traffic per gradient launch (PMC): fetch {fetch/1e9:.3f} GB, write {write/1e9:.4f} GB "
            f"({write_pred/1e9:.4f} GB at a trajectory's first/last launch, predictions included); "
            f"algorithmic {pmc['alg_bytes_per_launch']/1e9:.3f} GB\n\n")
    if fwd_fetch is not None:
        xb = bench["roofline"]["alg_bytes_per_launch"] - 4 * int(bench["config"]["n"]) * (
            1 if "network error once" in bench["roofline"].get("alg_bytes_basis", "") else int(bench["config"]["branches_per_gpu"]))
        fmean = statistics.mean(next(v for k, v in per_kernel.items() if fwd_fetch[0] in k)) if any(fwd_fetch[0] in k for k in per_kernel) else None
        f.write(f"Forward-only launch ({fwd_fetch[0]}, PMC): fetch {fwd_fetch[1]/1e9:.3f} GB per launch against "
                f"{xb/1e9:.3f} GB of 2-bit genotypes"
                + (f"; timed-trajectory mean {fmean:.4f} ms = {xb / (fmean * 1e-3) / 1e9:.0f} GB/s = "
                   f"{xb / (fmean * 1e-3) / 8e12:.3f} of 8 TB/s" if fmean else "") + "\n\n")
    f.write(f"achieved (algorithmic bytes / median launch): "
            f"{pmc['alg_bytes_per_launch'] / (statistics.median(dur) * 1e-3) / 1e9:.0f} GB/s\n\n")
    if "mfma" in pmc:
        m = pmc["mfma"]
        f.write("MFMA pass (median per gradient launch): " +
                ", ".join(f"{k} {v:.4g}" for k, v in m["counters_median_per_launch"].items()) +
                f"; matrix-pipe busy fraction {m['mfma_busy_per_simd_cycle']:.3f} per SIMD-cycle "
                f"({m['mfma_busy_per_cu_cycle']:.3f} per CU-cycle)\n\n")
    f.write("Full per-kernel stats of the command (all launches, setup included): "
            f"`{tag}_kernel_stats.csv`.\n")
print(open(os.path.join(prof, f"{tag}_summary.md")).read())

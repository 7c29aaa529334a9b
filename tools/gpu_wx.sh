#!/bin/bash
# wx: parity subset + C5 bench (f32, bf16), output gpurun_out/wx
set -o pipefail
mkdir -p gpurun_out/wx
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wx/pytest.txt 2>&1 || { tail -40 gpurun_out/wx/pytest.txt; exit 1; }
tail -2 gpurun_out/wx/pytest.txt
for bf in "" "--hidden-bf16"; do
  timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline $bf > gpurun_out/wx/c5$bf.json 2> gpurun_out/wx/c5$bf.err || { tail -5 gpurun_out/wx/c5$bf.err; exit 1; }
  python3 -c "import json;b=json.load(open('gpurun_out/wx/c5$bf.json'));r=b['roofline'];print('c5$bf',round(b['value'],2),round(r['kernel_ms'],2),round(r['achieved'],1),round(r['frac'],3),b['accept_rate'])"
done

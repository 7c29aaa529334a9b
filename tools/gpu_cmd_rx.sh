mkdir -p gpurun_out/rx
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/rx/pytest.txt 2>&1; echo pytest=$?; tail -3 gpurun_out/rx/pytest.txt
timeout -k 10 120 python tools/kbench.py --branches 1000 --tag rx || exit 1
for a in 1 15; do BANN_LIB=rs-bann_amd/abl/librsbann_amd_abl$a.so timeout -k 10 120 python tools/kbench.py --branches 1000 --tag rx_abl$a || exit 1; done
./tools/pmc.sh rx --branches 1000 || exit 1

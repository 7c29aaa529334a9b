set -o pipefail
export VARIANTS="ilp mcl" REPS=2
TAG=ab_fx NB=1000 ITERS=30 KB="" bash tools/gpu_kab.sh && \
TAG=ab_wx NB=4000 ITERS=20 KB="--n 100000 --m 125 --widths 32,32,1" bash tools/gpu_kab.sh && \
TAG=ab_gx NB=1000 ITERS=5 KB="--n 50000 --m 500 --widths 250,250,1" bash tools/gpu_kab.sh

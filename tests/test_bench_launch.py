"""bench.py's own N-rank launch (CPU, gloo): `python bench.py --gpus 2` run
directly starts torch.distributed.run as a child process (no exec, nothing on
the GPU in the parent); with --check-launch every rank takes its
marker-balanced shard and runs the library's residual exchange step
(bann_residual_update_host, the exchange bann_exchange_residual performs for a
callback communicator), and rank 0's JSON line comes back through the parent."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args):
    env = dict(os.environ, BANN_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout   # ONE JSON line, rank 0's
    return json.loads(lines[0]), p.stderr


def test_bench_launches_two_ranks():
    out, err = _run(["--gpus", "2", "--check-launch"])
    assert "launching 2 ranks" in err
    assert out["n_gpus"] == 2 and out["parallelism"] == "branch-shard x2"
    assert out["ranks"] == [0, 1]
    assert out["shards"] == [[0, 500], [500, 1000]]
    assert out["exchange_max_err"] == 0.0


def test_bench_single_rank_runs_in_process():
    out, err = _run(["--gpus", "1", "--check-launch"])
    assert "launching" not in err
    assert out["n_gpus"] == 1 and out["ranks"] == [0] and out["shards"] == [[0, 1000]]


def test_step_factor_rule():
    """the Izmailov factor c fixes the trajectory length L eps (ridge_ard.rs:70-117):
    below the L a line was tuned at, bench.py keeps the tuned step size
    (c = c_ref L / L_ref), above it the tuned trajectory length (c = c_ref)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    f = bench.default_step_factor
    assert f("c3", "branch", False, 20) == 1.0 and f("c3", "branch", False, 100) == 1.0
    assert abs(f("c3", "branch", False, 10) - 0.5) < 1e-12
    assert abs(f("c5", "branch", False, 10) - 0.05) < 1e-12 and abs(f("c5", "branch", False, 20) - 0.1) < 1e-12
    assert abs(f("c5", "branch", True, 10) - 0.01) < 1e-12
    assert abs(f("c3", "network", False, 20) - 0.5) < 1e-12 and abs(f("c3", "network", False, 10) - 0.25) < 1e-12
    # without the common-mode step rule the joint state's stiff mode caps the factor
    assert abs(f("c3", "network", False, 20, "off") - 0.11) < 1e-12
    assert abs(f("c3def", "branch", False, 4) - 0.008) < 1e-12 and f("c3def", "branch", False, 20) == 0.02
    # C5's joint network state, tuned on MI355X: 0.02 with the rule, 0.0005 without
    assert abs(f("c5", "network", False, 20) - 0.02) < 1e-15 and abs(f("c5", "network", True, 20) - 0.01) < 1e-15
    assert abs(f("c5", "network", False, 20, "off") - 0.0005) < 1e-15
    # an untuned line: the branch sampler's factor, one tenth for the joint network state
    assert abs(f("c2", "network", False, 20) - 0.1) < 1e-12

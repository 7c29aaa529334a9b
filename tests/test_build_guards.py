"""Build-time guards for the hand-counted memory waits of the fxl kernel.

k_fused_grad_fxl<NL <= 3, ACT, FULL = 1> loads its W0-digit operands with inline
asm and waits on them with hand-counted ``s_waitcnt vmcnt`` (kernels_fx.hip).  A
register spill of such an operand while its load is in flight would store
garbage, so those instantiations must compile without VGPR spills.  (CPU test:
hipcc cross-compiles gfx950 here.)"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "rs-bann_amd", "csrc", "kernels_fx.hip")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_counted_fxl_instantiations_do_not_spill(tmp_path):
    out = subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                          "-c", SRC, "-o", str(tmp_path / "k.o"), "-Rpass-analysis=kernel-resource-usage"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    spills, name = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"VGPRs Spill: (\d+)", line)
        if m and name:
            spills[name] = int(m.group(1))
    counted = [k for k in spills if re.match(r"_Z16k_fused_grad_fxlILi[23]ELi\dELi1ELi8E", k)]
    assert len(counted) == 10, counted
    assert all(spills[k] == 0 for k in counted), {k: spills[k] for k in counted}
    # 4 chunks per wave: the digit operands stay in registers for the whole item
    resident = [k for k in spills if re.match(r"_Z16k_fused_grad_fxlILi[23]ELi\dELi[01]ELi4E", k)]
    assert len(resident) == 20, resident
    assert all(spills[k] == 0 for k in resident), {k: spills[k] for k in resident}
    fx = [k for k in spills if k.startswith("_Z15k_fused_grad_fx")]
    assert fx and all(spills[k] == 0 for k in fx), {k: spills[k] for k in fx}
    fwd = [k for k in spills if k.startswith("_Z12k_forward_fx")]
    assert fwd and all(spills[k] == 0 for k in fwd), {k: spills[k] for k in fwd}


def test_production_kernels_carry_no_profiling_switches():
    """the ablation / stamp switches live in the profiling copy
    (tools/archive/profiling/kernels_fx_ablate.hip), not in the shipped kernels"""
    for f in os.listdir(os.path.dirname(SRC)):
        if f.endswith((".hip", ".h", ".cpp")):
            txt = open(os.path.join(os.path.dirname(SRC), f)).read()
            assert "#if BANN_ABLATE" not in txt and "FX_STAMP" not in txt, f

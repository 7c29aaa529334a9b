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


def test_production_build_sets_no_profiling_switches():
    """the fx kernel's profiling switches (FX_STAMPS phase stamps, FX_ABL ablations;
    tools/build_ab.sh builds variant libraries with them) default to 0 in the source
    and the product build (Makefile, __graft_entry__.build) defines none of them"""
    txt = open(SRC).read()
    for sw in ("FX_STAMPS", "FX_ABL"):
        assert f"#ifndef {sw}\n#define {sw} 0\n#endif" in txt, sw
    mk = open(os.path.join(os.path.dirname(SRC), "Makefile")).read()
    entry = open(os.path.join(ROOT, "__graft_entry__.py")).read()
    assert "-DFX_" not in mk and "-DFX_" not in entry and "BANN_ABLATE" not in mk

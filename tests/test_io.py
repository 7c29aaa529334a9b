"""Files on either side of the path, through the library's host-only C ABI (CPU):
PLINK dims (io/dims.rs), external / uniform groupings (group/external.rs,
group/uniform.rs), bincode .phen phenotypes (data/phenotypes.rs).  Fixtures
are the reference's own test data files (tests/golden/plink, copied from
resources/test)."""
import os
import struct

import numpy as np
import pytest

from bann import BannError
from bann.io import bed_dims, read_grouping, read_phen, uniform_grouping, write_phen

PLINK = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "plink")


def test_bed_dims_from_fam_bim_and_dims_file():
    assert bed_dims(os.path.join(PLINK, "small")) == (20, 11)      # resources/test/README.md: n = 20, m = 11
    assert bed_dims(os.path.join(PLINK, "random")) == (100, 20)    # random.dims
    with pytest.raises(BannError):
        bed_dims(os.path.join(PLINK, "missing"))


def test_external_grouping_small():
    gs = read_grouping(os.path.join(PLINK, "small.gene_grouping"))
    assert [g.tolist() for g in gs] == [[0, 1, 2, 3], [1, 2, 3, 5], [5, 6, 7, 8, 9, 10]]   # overlapping groups


def test_external_grouping_rejects_gaps(tmp_path):
    p = tmp_path / "g.txt"
    p.write_text("0 0\n1 2\n")   # group 1 missing (external.rs:46-49)
    with pytest.raises(BannError):
        read_grouping(str(p))


def test_uniform_grouping():
    gs = uniform_grouping(3, 4)
    assert [g.tolist() for g in gs] == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9, 10, 11]]


def test_phen_roundtrip_is_bincode(tmp_path):
    y = np.array([0.5, -1.25, 3.0, 7.75], np.float32)
    p = str(tmp_path / "y.phen")
    write_phen(p, y)
    raw = open(p, "rb").read()
    assert raw[:8] == struct.pack("<Q", 4) and raw[8:] == y.tobytes()   # bincode Vec<f32>: u64 length + LE f32
    assert np.array_equal(read_phen(p), y)

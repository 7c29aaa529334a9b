"""Files on either side of the hot path, through the library's host-only C ABI
(no device needed): PLINK dims, marker groupings, bincode phenotypes.

  bed_dims            BedDims (io/dims.rs:15-34)
  read_grouping       ExternalGrouping::from_file (group/external.rs:15-60)
  uniform_grouping    UniformGrouping::new (group/uniform.rs:11-23)
  read_phen/write_phen Phenotypes::from_file / to_file (data/phenotypes.rs:28-36)
"""
from __future__ import annotations

import ctypes as C
from typing import List

import numpy as np

from ._lib import BannError, load_library


def _chk(rc, what):
    if rc != 0:
        raise BannError(rc, what)


def bed_dims(stem: str):
    """(n, num_markers) of a PLINK fileset stem: stem.dims, else the .fam / .bim line counts."""
    n, m = C.c_int64(), C.c_int64()
    _chk(load_library().bann_bed_dims(stem.encode(), C.byref(n), C.byref(m)), f"bann_bed_dims({stem})")
    return n.value, m.value


def read_grouping(path: str) -> List[np.ndarray]:
    """marker index lists of an external grouping file (one int32 array per group)."""
    lib = load_library()
    G, E = C.c_int32(), C.c_int64()
    _chk(lib.bann_grouping_read(path.encode(), C.byref(G), C.byref(E), None, None), f"bann_grouping_read({path})")
    off = np.zeros(G.value + 1, np.int64)
    mk = np.zeros(max(E.value, 1), np.int32)
    _chk(lib.bann_grouping_read(path.encode(), C.byref(G), C.byref(E), off.ctypes.data_as(C.POINTER(C.c_int64)),
                                mk.ctypes.data_as(C.POINTER(C.c_int32))), f"bann_grouping_read({path})")
    return [mk[off[g]:off[g + 1]].copy() for g in range(G.value)]


def uniform_grouping(num_groups: int, group_size: int) -> List[np.ndarray]:
    off = np.zeros(num_groups + 1, np.int64)
    mk = np.zeros(num_groups * group_size, np.int32)
    _chk(load_library().bann_grouping_uniform(num_groups, group_size, off.ctypes.data_as(C.POINTER(C.c_int64)),
                                              mk.ctypes.data_as(C.POINTER(C.c_int32))), "bann_grouping_uniform")
    return [mk[off[g]:off[g + 1]].copy() for g in range(num_groups)]


def read_phen(path: str) -> np.ndarray:
    lib = load_library()
    n = C.c_int64()
    _chk(lib.bann_phen_read(path.encode(), C.byref(n), None), f"bann_phen_read({path})")
    y = np.zeros(n.value, np.float32)
    _chk(lib.bann_phen_read(path.encode(), C.byref(n), y.ctypes.data_as(C.POINTER(C.c_float))),
         f"bann_phen_read({path})")
    return y


def write_phen(path: str, y) -> None:
    ya = np.ascontiguousarray(y, dtype=np.float32)
    _chk(load_library().bann_phen_write(path.encode(), ya.ctypes.data_as(C.POINTER(C.c_float)), ya.size),
         f"bann_phen_write({path})")

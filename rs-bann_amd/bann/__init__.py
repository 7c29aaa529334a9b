"""rs-bann_amd: MI355X-native branch-network HMC hot path (host-side mirror).

The compute lives in the in-tree HIP library ``rs-bann_amd/librsbann_amd.so``
(C ABI: ``include/bann.h``, ``include/bann_net.h``); this package only binds it.
"""
from ._lib import (ACTIVATIONS, HMC_STATUS, LIB_PATH, PRIORS, STEP_MODES, BannError, BannLibraryError,
                   load_library)
from .context import BannContext
from .net import MCMCConfig, Net

__all__ = ["BannContext", "Net", "MCMCConfig", "BannError", "BannLibraryError", "load_library", "LIB_PATH", "ACTIVATIONS", "PRIORS",
           "STEP_MODES", "HMC_STATUS"]

"""ldpcgputegra_amd -- MI355X-native layered min-sum LDPC decoder.

Drop-in for the decode path of boiseHPSim/ldpcGpuTegra
(CDecoder::decode(llr, hard, iters)); see DESIGN.md and INTEGRATION.md.
The compute path is the HIP library ``libldpc_mi355x.so`` (C-ABI in
include/ldpc_mi355x.h); this package is its host-side binding.
"""
from . import _lib
from ._lib import ALGO_MS, ALGO_NMS, ALGO_OMS, LdpcError, default_params
from .codes import Code, Table, available, load_table
from .decoder import (CDecoder, CDecoder_NMS_fixed_MI355X, CDecoder_OMS_fixed_MI355X, CreateDecoder, Decoder,
                      param_decoder, pinned_empty)

__all__ = [
    "ALGO_MS", "ALGO_NMS", "ALGO_OMS", "LdpcError", "default_params", "Code", "Table", "available",
    "load_table", "CDecoder", "CDecoder_OMS_fixed_MI355X", "CDecoder_NMS_fixed_MI355X", "CreateDecoder",
    "Decoder", "param_decoder", "pinned_empty",
]

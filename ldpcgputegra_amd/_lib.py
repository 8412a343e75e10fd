"""ctypes binding of the C-ABI in include/ldpc_mi355x.h.

The shared library is built in-tree (``ldpcgputegra_amd/libldpc_mi355x.so``,
see ``__graft_entry__.build``).  There is no fallback: if the library is
missing, importing the decoder raises -- the product path never silently
drops to a CPU implementation.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# LDPC_MI355X_LIB: an alternative build of the same library (kernel variants, tools/variants.sh)
LIB_PATH = os.environ.get("LDPC_MI355X_LIB") or os.path.join(_HERE, "libldpc_mi355x.so")

LDPC_OK, LDPC_EINVAL, LDPC_EUNSUPPORTED, LDPC_EDEVICE, LDPC_ENOMEM, LDPC_EIO = 0, -1, -2, -3, -4, -5
ALGO_OMS, ALGO_NMS, ALGO_MS = 0, 1, 2


def source_hash():
    """sha256 (16 hex digits) over the sources the library is built from
    (csrc/* and include/*): ties a committed measurement (profiles/traffic.json)
    to the exact kernel code it was taken on.  A variant library
    (LDPC_MI355X_LIB, tools/build_variant.sh) folds in its extra defines
    (the `.defines` stamp written beside it) -- or, without a stamp, its path --
    so a variant never reports the default build's hash."""
    import hashlib
    root = os.path.dirname(_HERE)
    h = hashlib.sha256()
    for d in (os.path.join(_HERE, "csrc"), os.path.join(root, "include")):
        for f in sorted(os.listdir(d)):
            fp = os.path.join(d, f)
            if os.path.isfile(fp):
                h.update(f.encode())
                with open(fp, "rb") as fh:
                    h.update(fh.read())
    if os.path.abspath(LIB_PATH) != os.path.abspath(os.path.join(_HERE, "libldpc_mi355x.so")):
        stamp = LIB_PATH + ".defines"
        if os.path.exists(stamp):
            with open(stamp, "rb") as fh:
                h.update(b"variant:" + fh.read())
        else:
            h.update(b"variant-path:" + os.path.abspath(LIB_PATH).encode())
    return h.hexdigest()[:16]


class LdpcError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__("%s (%d): %s" % (_strerror(status), status, msg))
        self.status = status


class ldpc_params(C.Structure):
    _fields_ = [
        ("algo", C.c_int), ("offset", C.c_int), ("factor", C.c_int), ("beta", C.c_float),
        ("var_min", C.c_int), ("var_max", C.c_int), ("msg_min", C.c_int), ("msg_max", C.c_int),
        ("early_term", C.c_int),
    ]


# name -> (restype, argtypes); every exported symbol of include/ldpc_mi355x.h
P = C.c_void_p
I = C.c_int
U64 = C.c_uint64
SIGNATURES = {
    "ldpc_params_default": (None, [C.POINTER(ldpc_params)]),
    "ldpc_strerror": (C.c_char_p, [I]),
    "ldpc_last_error": (C.c_char_p, []),
    "ldpc_abi_version": (I, []),
    "ldpc_device_count": (I, [C.POINTER(I)]),
    "ldpc_code_create": (I, [I, I, I, P, P, P, C.POINTER(P)]),
    "ldpc_code_from_dvbs2_table": (I, [I, I, I, P, P, C.POINTER(P)]),
    "ldpc_code_load": (I, [C.c_char_p, C.POINTER(P)]),
    "ldpc_code_info": (I, [P, C.POINTER(I), C.POINTER(I), C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
    "ldpc_code_edges": (I, [P, P, P, P]),
    "ldpc_code_plan_info": (I, [P, C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
    "ldpc_code_layer_info": (I, [P, C.POINTER(I), C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
    "ldpc_code_window_plan": (I, [P, I, I, P, P, I, C.POINTER(I)]),
    "ldpc_code_coop_plan": (I, [P, I, I, P, P, I, C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
    "ldpc_code_coop_plan_dist": (I, [P, I, I, I, P, P, I, C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
    "ldpc_code_coop3_lc_info": (I, [P] + [C.POINTER(I)] * 5),
    "ldpc_code_coop3_lc_banks": (I, [P, C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]),
    "ldpc_code_destroy": (None, [P]),
    "ldpc_ctx_create": (I, [P, I, I, C.POINTER(P)]),
    "ldpc_ctx_destroy": (None, [P]),
    "ldpc_ctx_stream": (I, [P, C.POINTER(P)]),
    "ldpc_ctx_set_kernel": (I, [P, I]),
    "ldpc_ctx_get_kernel": (I, [P, C.POINTER(I)]),
    "ldpc_ctx_last_kernel": (I, [P, C.POINTER(I)]),
    "ldpc_ctx_last_skipped": (I, [P, C.POINTER(I)]),
    "ldpc_ctx_last_et_stage": (I, [P, C.POINTER(I)]),
    "ldpc_ctx_profile": (I, [P, I]),
    "ldpc_ctx_kernel_time": (I, [P, C.POINTER(C.c_double), C.POINTER(I), I]),
    "ldpc_decode_i8": (I, [P, P, P, I, I, C.POINTER(ldpc_params)]),
    "ldpc_decode_f32": (I, [P, P, P, I, I, C.POINTER(ldpc_params)]),
    "ldpc_decode_i8_async": (I, [P, P, P, P, P, P, I, I, C.POINTER(ldpc_params)]),
    "ldpc_decode_f32_async": (I, [P, P, P, P, P, P, I, I, C.POINTER(ldpc_params)]),
    "ldpc_decode_i8_nm_async": (I, [P, P, P, C.c_size_t, P, P, P, I, I, C.POINTER(ldpc_params)]),
    "ldpc_mixed_create": (I, [P, I, I, I, C.POINTER(P)]),
    "ldpc_mixed_destroy": (None, [P]),
    "ldpc_decode_i8_mixed_async": (I, [P, P, P, P, P, P, I, I, C.POINTER(ldpc_params)]),
    "ldpc_mixed_last_kernel": (I, [P, I, C.POINTER(I)]),
    "ldpc_mixed_last_et_stage": (I, [P, I, C.POINTER(I)]),
    "ldpc_mixed_profile": (I, [P, I]),
    "ldpc_mixed_kernel_time": (I, [P, I, C.POINTER(C.c_double), C.POINTER(I), I]),
    "ldpc_dvbs2_encode": (I, [P, P, P, I]),
    "ldpc_awgn_sigma": (C.c_double, [C.c_double, C.c_double]),
    "ldpc_awgn_i8_table": (I, [C.c_double, I, I, P]),
    "ldpc_awgn_sigma_ex": (C.c_double, [C.c_double, C.c_double, I]),
    "ldpc_awgn_i8_table_ex": (I, [C.c_double, C.c_double, C.c_double, I, I, P]),
    "ldpc_awgn_i8_host": (I, [I, I, U64, U64, P, P, P]),
    "ldpc_awgn_i8_async": (I, [P, P, P, I, U64, U64, P, P]),
    "ldpc_count_errors_async": (I, [P, P, P, I, I, P, P]),
    "ldpc_decode_i8_count_async": (I, [P, P, P, P, P, P, I, I, C.POINTER(ldpc_params), I, P, P]),
    "ldpc_decode_f32_count_async": (I, [P, P, P, P, P, P, I, I, C.POINTER(ldpc_params), I, P, P]),
    "ldpc_quantize_f32_i8_async": (I, [P, P, P, P, C.c_long, I, I, I]),
    "ldpc_quantize_f32_i8": (I, [P, P, P, C.c_long, I, I, I]),
    "ldpc_decode_i8_host_async": (I, [P, P, P, P, I, I, C.POINTER(ldpc_params)]),
    "ldpc_decode_f32_host_async": (I, [P, P, P, P, I, I, C.POINTER(ldpc_params)]),
    "ldpc_ctx_synchronize": (I, [P]),
    "ldpc_host_alloc": (I, [C.POINTER(P), C.c_size_t]),
    "ldpc_host_free": (None, [P]),
}

_lib = None


def lib():
    """Load libldpc_mi355x.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        # One process holds one HIP runtime: libamdhip64.so.7 is resolved by
        # soname, so whichever copy loads first (ROCm's, or the one bundled in
        # PyTorch's wheel) serves everybody.  When PyTorch is installed we let
        # it load first, so the device tensors handed to us and our kernels
        # share its runtime (loading ours first leaves torch.cuda unusable).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError("libldpc_mi355x.so not built: run `python -c 'import __graft_entry__ as g; g.build()'`"
                              " (expected at %s)" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        missing = [name for name in SIGNATURES if not hasattr(L, name)]
        if missing and os.environ.get("LDPC_AB_OLD_LIB") != "1":
            raise ImportError("%s lacks entry points of include/ldpc_mi355x.h (stale build?): %s"
                              % (LIB_PATH, ", ".join(missing)))
        for name, (res, args) in SIGNATURES.items():
            if name in missing:
                continue   # LDPC_AB_OLD_LIB=1 (tools/ab.sh's older experiment builds): left unbound
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _strerror(status):
    try:
        return lib().ldpc_strerror(status).decode()
    except Exception:  # pragma: no cover
        return "error"


def check(status):
    if status != LDPC_OK:
        raise LdpcError(status, lib().ldpc_last_error().decode())
    return status


def default_params(**kw):
    p = ldpc_params()
    lib().ldpc_params_default(C.byref(p))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise TypeError("unknown ldpc_params field %r" % k)
        setattr(p, k, v)
    return p

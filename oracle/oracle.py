"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

* ``liboracle.so``       -- our scalar restatement (ldpc_oracle.c)
* ``_ref/<code>/libref.so`` -- the reference's own SSE decoders compiled from
  /root/reference (oracle/Makefile); present only where it was built.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product (ldpcgputegra_amd) never does.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_DIR = os.path.join(HERE, "_ref")

# reference Constantes directory for each shipped code name
REF_CODE_DIRS = {
    "576x288": "576x288", "1944x972": "1944x972", "2304x1152": "2304x1152", "2048x384": "2048x384",
    "4000x2000": "4000x2000", "dvbs2_r1_2": "64800x32400.dvb-s2", "dvbs2_r8_9": "64800x7200.dvb-s2",
    "dvbs2_r9_10": "64800x6480.dvb-s2",
}

OMS, NMS = 0, 1


class _Code(C.Structure):
    _fields_ = [("n", C.c_int), ("m", C.c_int), ("e", C.c_int), ("n_groups", C.c_int),
                ("group_deg", C.POINTER(C.c_int)), ("group_cnt", C.POINTER(C.c_int)),
                ("edge_var", C.POINTER(C.c_uint32))]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "oracle"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = C.CDLL(ORACLE_SO)
        P = C.c_void_p
        L.oracle_decode_i8.argtypes = [C.POINTER(_Code), P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.c_int, C.c_int, C.c_int, P]
        L.oracle_decode_f32.argtypes = [C.POINTER(_Code), P, P, P, C.c_int, C.c_int, C.c_int, C.c_float, C.c_int, P]
        L.oracle_decode_i8_mt.argtypes = [C.POINTER(_Code), P, P, C.c_int, C.c_int, C.c_int, C.c_int]
        L.oracle_decode_i8_mt_ex.argtypes = [C.POINTER(_Code), P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                             P, C.c_int]
        L.oracle_decode_f32_mt.argtypes = [C.POINTER(_Code), P, P, P, C.c_int, C.c_int, C.c_int, C.c_float, C.c_int,
                                           P, C.c_int]
        L.oracle_quantize.argtypes = [P, P, C.c_long, C.c_int, C.c_int, C.c_int]
        L.oracle_quantize.restype = None
        L.oracle_syndrome.argtypes = [C.POINTER(_Code), P]
        _lib = L
    return _lib


class OracleCode:
    def __init__(self, table):
        self.table = table
        self._gd = np.ascontiguousarray(table.group_deg, dtype=np.int32)
        self._gc = np.ascontiguousarray(table.group_cnt, dtype=np.int32)
        self._ev = np.ascontiguousarray(table.edge_var, dtype=np.uint32)
        self.c = _Code(table.n, table.m, table.e, len(table.groups),
                       self._gd.ctypes.data_as(C.POINTER(C.c_int)), self._gc.ctypes.data_as(C.POINTER(C.c_int)),
                       self._ev.ctypes.data_as(C.POINTER(C.c_uint32)))


def host_threads():
    """Threads for the oracle on this host: the CPU share the process may
    use (the GPU box grants 16 CPUs of a larger machine through its cgroup)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def decode_i8(table, llr, iters, algo=OMS, param=1, var_min=-127, var_max=127, msg_max=31, early_term=False,
              return_soft=False, threads=1):
    oc = OracleCode(table)
    llr = np.ascontiguousarray(llr, dtype=np.int8).reshape(-1, table.n)
    B = llr.shape[0]
    hard = np.empty_like(llr, dtype=np.uint8)
    soft = np.empty_like(llr) if return_soft else None
    its = np.empty(B, dtype=np.int32)
    if threads > 1 and var_min == -127 and var_max == 127 and msg_max == 31:
        rc = lib().oracle_decode_i8_mt_ex(C.byref(oc.c), llr.ctypes.data, hard.ctypes.data,
                                          soft.ctypes.data if soft is not None else None, B, iters, algo, param,
                                          int(early_term), its.ctypes.data, threads)
    else:
        rc = lib().oracle_decode_i8(C.byref(oc.c), llr.ctypes.data, hard.ctypes.data,
                                    soft.ctypes.data if soft is not None else None, B, iters, algo, param, var_min,
                                    var_max, msg_max, int(early_term), its.ctypes.data)
    if rc != 0:
        raise ValueError("oracle rejected parameters")
    if return_soft:
        return hard, soft, its
    return hard


def decode_f32(table, llr, iters, algo=OMS, beta=0.0, early_term=False, threads=1):
    oc = OracleCode(table)
    llr = np.ascontiguousarray(llr, dtype=np.float32).reshape(-1, table.n)
    B = llr.shape[0]
    hard = np.empty(llr.shape, dtype=np.uint8)
    soft = np.empty_like(llr)
    its = np.empty(B, dtype=np.int32)
    if threads > 1:
        rc = lib().oracle_decode_f32_mt(C.byref(oc.c), llr.ctypes.data, hard.ctypes.data, soft.ctypes.data, B,
                                        iters, algo, beta, int(early_term), its.ctypes.data, threads)
    else:
        rc = lib().oracle_decode_f32(C.byref(oc.c), llr.ctypes.data, hard.ctypes.data, soft.ctypes.data, B, iters,
                                     algo, beta, int(early_term), its.ctypes.data)
    if rc != 0:
        raise ValueError("oracle rejected parameters")
    return hard, soft, its


def decode_i8_mt(table, llr, iters, offset=1, threads=1):
    oc = OracleCode(table)
    llr = np.ascontiguousarray(llr, dtype=np.int8).reshape(-1, table.n)
    hard = np.empty_like(llr, dtype=np.uint8)
    rc = lib().oracle_decode_i8_mt(C.byref(oc.c), llr.ctypes.data, hard.ctypes.data, llr.shape[0], iters, offset,
                                   threads)
    assert rc == 0
    return hard


def quantize(y, factor=8, sat_neg=-31, sat_pos=31):
    y = np.ascontiguousarray(y, dtype=np.float32)
    q = np.empty(y.shape, dtype=np.int8)
    lib().oracle_quantize(y.ctypes.data, q.ctypes.data, y.size, factor, sat_neg, sat_pos)
    return q


# ---- the reference itself (built here only; travels to the GPU box) -------

def ref_available(code_name):
    d = REF_CODE_DIRS.get(code_name)
    return d is not None and os.path.exists(os.path.join(REF_DIR, d, "libref.so"))


_ref_libs = {}


def ref_lib(code_name):
    if code_name not in _ref_libs:
        path = os.path.join(REF_DIR, REF_CODE_DIRS[code_name], "libref.so")
        L = C.CDLL(path)
        P = C.c_void_p
        L.ref_decode.argtypes = [P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        L.ref_decode_mt.argtypes = [P, P, C.c_int, C.c_int, C.c_int, C.c_int]
        L.ref_code_info.argtypes = [C.POINTER(C.c_int)] * 3
        _ref_libs[code_name] = L
    return _ref_libs[code_name]


def ref_decode(code_name, llr, iters, algo=OMS, param=1, vmin=-127, vmax=127, mmin=-31, mmax=31):
    L = ref_lib(code_name)
    n, m, e = C.c_int(), C.c_int(), C.c_int()
    L.ref_code_info(C.byref(n), C.byref(m), C.byref(e))
    llr = np.ascontiguousarray(llr, dtype=np.int8).reshape(-1, n.value)
    B = llr.shape[0]
    assert B % 16 == 0, "the reference decodes 16 frames per call"
    hard = np.empty_like(llr, dtype=np.uint8)
    rc = L.ref_decode(llr.ctypes.data, hard.ctypes.data, B, iters, algo, param, vmin, vmax, mmin, mmax)
    assert rc == 0
    return hard


def ref_decode_mt(code_name, llr, iters, offset=1, threads=1):
    L = ref_lib(code_name)
    llr = np.ascontiguousarray(llr, dtype=np.int8)
    B = llr.shape[0]
    hard = np.empty_like(llr, dtype=np.uint8)
    rc = L.ref_decode_mt(llr.ctypes.data, hard.ctypes.data, B, iters, offset, threads)
    assert rc == 0
    return hard

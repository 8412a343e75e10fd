"""LDPC code registry: runtime H tables.

Replaces the reference's compile-time code selection (``#include`` of one
``Constantes/<code>/constantes_sse.h``, code/x86/Constantes/constantes_sse.h:1-2,
and ``#define CODE 1200`` in code/gpu_fixed/matrix/code.h:1): any shipped code
is opened by name at run time.

Two table formats live in ``ldpcgputegra_amd/codes/``:

* ``<name>.ldpc``  -- LDPCH001 binary: magic, u32 n, m, e, n_groups,
  n_groups x (u32 degree, u32 count), e x u32 variable index (layered order).
* ``dvbs2_*.txt``  -- DVB-S2 Annex-B address tables; H is rebuilt by the C
  library (``ldpc_code_from_dvbs2_table``) with the reference's layered order.

``load_table`` is a pure-numpy reader used by tests and the oracle;
``Code`` wraps the C-ABI handle used by the decoder.
"""
import ctypes as C
import os
import struct

import numpy as np

from . import _lib

CODE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "codes")

ALIASES = {
    "dvbs2": "dvbs2_r1_2",
    "64800x32400": "dvbs2_r1_2",
    "64800x21600": "dvbs2_r2_3",
    "64800x7200": "dvbs2_r8_9",
    "64800x6480": "dvbs2_r9_10",
    "80211n_648": "648x324",
}


def code_path(name):
    name = ALIASES.get(name, name)
    for ext in (".ldpc", ".txt"):
        p = os.path.join(CODE_DIR, name + ext)
        if os.path.exists(p):
            return p
    if os.path.exists(name):
        return name
    raise FileNotFoundError("unknown LDPC code %r (see %s)" % (name, CODE_DIR))


def available():
    out = []
    for f in sorted(os.listdir(CODE_DIR)):
        if f.endswith(".ldpc") or (f.startswith("dvbs2") and f.endswith(".txt")):
            out.append(os.path.splitext(f)[0])
    return out


class Table:
    """Plain numpy view of a layered H (n, m, groups, edge_var)."""

    def __init__(self, n, m, groups, edge_var):
        self.n, self.m = int(n), int(m)
        self.groups = [(int(d), int(c)) for d, c in groups]
        self.edge_var = np.ascontiguousarray(edge_var, dtype=np.uint32)
        self.e = int(self.edge_var.size)
        assert sum(d * c for d, c in self.groups) == self.e
        assert sum(c for _, c in self.groups) == self.m

    @property
    def k_info(self):
        return self.n - self.m

    @property
    def group_deg(self):
        return np.array([d for d, _ in self.groups], dtype=np.int32)

    @property
    def group_cnt(self):
        return np.array([c for _, c in self.groups], dtype=np.int32)

    def checks(self):
        """Yield (group index, variable array) per check in layered order."""
        pos = 0
        for g, (d, c) in enumerate(self.groups):
            for _ in range(c):
                yield g, self.edge_var[pos:pos + d]
                pos += d

    def syndrome(self, hard):
        """Number of unsatisfied checks of 0/1 array ``hard`` [N] or [B, N]."""
        hard = np.asarray(hard, dtype=np.uint8)
        pos, bad = 0, 0
        for d, c in self.groups:
            idx = self.edge_var[pos:pos + d * c].reshape(c, d)
            par = np.bitwise_xor.reduce(hard[..., idx], axis=-1)
            bad = bad + par.sum(axis=-1)
            pos += d * c
        return bad


def _dvbs2_from_text(path):
    n = k = None
    rows = []
    for line in open(path):
        line = line.strip()
        if not line:
            continue
        if line.startswith("#"):
            if "N=" in line and "K=" in line:
                toks = dict(t.split("=") for t in line[1:].split() if "=" in t)
                n, k = int(toks["N"]), int(toks["K"])
            continue
        rows.append([int(x) for x in line.split()])
    m = n - k
    q = m // 360
    info = [[] for _ in range(m)]
    for g, row in enumerate(rows):
        for kk in range(360):
            v = 360 * g + kk
            for x in row:
                info[(x + kk * q) % m].append(v)
    edges, groups = [], []
    for idx in range(m):
        r = (idx + 1) % m
        lst = sorted(info[r]) + ([k + r - 1, k + r] if r > 0 else [k])
        edges.extend(lst)
        if groups and groups[-1][0] == len(lst):
            groups[-1][1] += 1
        else:
            groups.append([len(lst), 1])
    return Table(n, m, groups, np.array(edges, dtype=np.uint32))


def load_table(name):
    """Pure-numpy table reader (no C library needed)."""
    path = code_path(name)
    data = open(path, "rb").read()
    if data[:8] == b"LDPCH001":
        n, m, e, ng = struct.unpack_from("<IIII", data, 8)
        groups = [struct.unpack_from("<II", data, 24 + 8 * g) for g in range(ng)]
        ev = np.frombuffer(data, dtype="<u4", count=e, offset=24 + 8 * ng)
        return Table(n, m, groups, ev)
    return _dvbs2_from_text(path)


class Code:
    """C-ABI ``ldpc_code`` handle (immutable, shareable across contexts)."""

    def __init__(self, name_or_table):
        L = _lib.lib()
        h = C.c_void_p()
        if isinstance(name_or_table, Table):
            t = name_or_table
            gd, gc = t.group_deg, t.group_cnt
            _lib.check(L.ldpc_code_create(t.n, t.m, len(t.groups), gd.ctypes.data, gc.ctypes.data,
                                          t.edge_var.ctypes.data, C.byref(h)))
            self.name = "custom"
        else:
            _lib.check(L.ldpc_code_load(code_path(name_or_table).encode(), C.byref(h)))
            self.name = ALIASES.get(name_or_table, name_or_table)
        self._h = h
        n, m, e, ng, md = (C.c_int() for _ in range(5))
        _lib.check(L.ldpc_code_info(h, C.byref(n), C.byref(m), C.byref(e), C.byref(ng), C.byref(md)))
        self.n, self.m, self.e, self.n_groups, self.max_deg = n.value, m.value, e.value, ng.value, md.value

    @property
    def handle(self):
        return self._h

    @property
    def k_info(self):
        return self.n - self.m

    def table(self):
        L = _lib.lib()
        ev = np.empty(self.e, dtype=np.uint32)
        gd = np.empty(self.n_groups, dtype=np.int32)
        gc = np.empty(self.n_groups, dtype=np.int32)
        _lib.check(L.ldpc_code_edges(self._h, ev.ctypes.data, gd.ctypes.data, gc.ctypes.data))
        return Table(self.n, self.m, list(zip(gd, gc)), ev)

    def plan_info(self):
        s, w, hz = C.c_int(), C.c_int(), C.c_int()
        _lib.check(_lib.lib().ldpc_code_plan_info(self._h, C.byref(s), C.byref(w), C.byref(hz)))
        return dict(staircase=bool(s.value), n_windows=w.value, min_hazard=hz.value, windowed=w.value > 0)

    def layer_info(self):
        """Layer plan of the LDS-resident kernel (kernel 7)."""
        nl, w, i8, f32 = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        _lib.check(_lib.lib().ldpc_code_layer_info(self._h, C.byref(nl), C.byref(w), C.byref(i8), C.byref(f32)))
        return dict(n_layers=nl.value, max_width=w.value, lds_i8=bool(i8.value), lds_f32=bool(f32.value))

    def encode(self, info):
        """DVB-S2 IRA encoding of info bits [batch, K] -> codewords [batch, N]."""
        info = np.ascontiguousarray(info, dtype=np.uint8).reshape(-1, self.k_info)
        cw = np.empty((info.shape[0], self.n), dtype=np.uint8)
        _lib.check(_lib.lib().ldpc_dvbs2_encode(self._h, info.ctypes.data, cw.ctypes.data, info.shape[0]))
        return cw

    def window_plan(self, S, P):
        """[(first check, count)] of the windowed2 schedule (empty if none)."""
        L = _lib.lib()
        n = C.c_int()
        _lib.check(L.ldpc_code_window_plan(self._h, S, P, None, None, 0, C.byref(n)))
        first = np.empty(max(n.value, 1), dtype=np.int32)
        count = np.empty(max(n.value, 1), dtype=np.int32)
        _lib.check(L.ldpc_code_window_plan(self._h, S, P, first.ctypes.data, count.ctypes.data, n.value,
                                           C.byref(n)))
        return list(zip(first[:n.value].tolist(), count[:n.value].tolist()))

    def coop_plan(self, S=28, R=3, dist=1):
        """Schedule of the workgroup-cooperative kernels (dist 1: coop, 2:
        coop2): dict(windows=[(first, count)], tail=window index of the tail
        check, n_fwd=forwarded reads per iteration); None when the code has no
        such schedule."""
        L = _lib.lib()
        n, t, f = C.c_int(), C.c_int(), C.c_int()
        _lib.check(L.ldpc_code_coop_plan_dist(self._h, S, R, dist, None, None, 0, C.byref(n), C.byref(t),
                                              C.byref(f)))
        if n.value == 0:
            return None
        first = np.empty(n.value, dtype=np.int32)
        count = np.empty(n.value, dtype=np.int32)
        _lib.check(L.ldpc_code_coop_plan_dist(self._h, S, R, dist, first.ctypes.data, count.ctypes.data, n.value,
                                              C.byref(n), C.byref(t), C.byref(f)))
        return dict(windows=list(zip(first.tolist(), count.tolist())), tail=t.value, n_fwd=f.value)

    def coop3_line_cache(self):
        """Line-cache plan of the coop3 kernel (kernel 8): dict(slots,
        max_slots, residencies, prologue, epilogue); None when the code has no
        coop3 schedule."""
        v = [C.c_int() for _ in range(5)]
        _lib.check(_lib.lib().ldpc_code_coop3_lc_info(self._h, *[C.byref(x) for x in v]))
        if v[0].value == 0:
            return None
        return dict(zip(("slots", "max_slots", "residencies", "prologue", "epilogue"), (x.value for x in v)))

    def coop3_lc_banks(self):
        """Modelled extra LDS cycles per iteration and workgroup of coop3's
        line-cache pre reads / post writes: dict(swizzled=..., plain=...)
        (the planner's XOR swizzle vs every line unswizzled)."""
        a, b = C.c_longlong(), C.c_longlong()
        _lib.check(_lib.lib().ldpc_code_coop3_lc_banks(self._h, C.byref(a), C.byref(b)))
        return dict(swizzled=a.value, plain=b.value)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib._lib.ldpc_code_destroy(h)
            self._h = None

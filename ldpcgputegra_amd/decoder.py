"""Host-side mirror of the reference decoder interface, on the MI355X C-ABI.

Reference interface (code/x86/CDecoder/template/CDecoder.h:28-40,
CDecoder_fixed.h:30-44, OMS/CDecoder_OMS_fixed_SSE.h, NMS/...,
DecoderLibrary.h:44-134)::

    CDecoder*  CreateDecoder(type, arch, format, p_decoder, vMin, vMax, mMin, mMax)
    decoder->setOffset(k) / setFactor(k) / setVarRange / setMsgRange
    decoder->decode(char llr[16*N], char hard[16*N], int iterations)

Here ``CreateDecoder(..., arch="mi355x")`` returns an object with the same
methods and argument meaning; ``decode`` fills ``hard`` in place (0/1 per bit,
frame-major) like the reference.  Errors the reference handles with
``printf + exit(0)`` raise ``LdpcError`` instead.

``Decoder`` is the batch API used by tests and bench.py: any batch size,
host numpy arrays or device tensors (``*_device`` methods take torch tensors
on the GPU and enqueue on the current stream without synchronising).
"""
import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from .codes import Code

def pinned_empty(shape, dtype):
    """numpy array in page-locked host memory (ldpc_host_alloc, the
    reference's CUDA_MALLOC_HOST): the host-buffer decodes copy it by DMA,
    overlapped with the decodes of the other chunks.  Freed with the array."""
    import weakref
    dt = np.dtype(dtype)
    nbytes = int(np.prod(shape)) * dt.itemsize
    ptr = C.c_void_p()
    _lib.check(_lib.lib().ldpc_host_alloc(C.byref(ptr), max(nbytes, 1)))
    buf = (C.c_char * max(nbytes, 1)).from_address(ptr.value)
    weakref.finalize(buf, _lib.lib().ldpc_host_free, ptr)
    return np.frombuffer(buf, dtype=dt, count=int(np.prod(shape))).reshape(shape)


class Decoder:
    """One C-ABI decoder context (device scratch for ``max_batch`` codewords)."""

    def __init__(self, code, device=0, max_batch=4096, kernel=0):
        self.code = code if isinstance(code, Code) else Code(code)
        self.device = device
        self.max_batch = max_batch
        h = C.c_void_p()
        _lib.check(_lib.lib().ldpc_ctx_create(self.code.handle, device, max_batch, C.byref(h)))
        self._ctx = h
        self._pending = []   # (llr, hard) of queued host-buffer decodes, alive until synchronize()
        if kernel:
            self.set_kernel(kernel)

    # -- configuration
    def set_kernel(self, kernel):
        """0 = auto, 1 = generic (per-edge messages), 2 = windowed, 3 =
        windowed2 (S = 16), 5 = workgroup-cooperative DVB-S2 kernel (coop),
        7 = LDS-resident short-code kernel (int8 and float), 8 = coop3 (slab waves
        doing pre + post, i16 chain; the DVB-S2 r1/2 default), 9 = ldsep
        (edge-parallel float for short QC codes; the float default where it fits),
        11 = stairf (float staircase codes, DVB-S2: the float default for them,
        with or without early termination -- with it, one launch per iteration
        plus a syndrome pass, as include/ldpc_mi355x.h states).  4 and 6 (windowed2 S = 32, coop2) were
        superseded and removed."""
        _lib.check(_lib.lib().ldpc_ctx_set_kernel(self._ctx, int(kernel)))

    @property
    def kernel(self):
        k = C.c_int()
        _lib.check(_lib.lib().ldpc_ctx_get_kernel(self._ctx, C.byref(k)))
        return k.value

    def profile(self, enable=True):
        """Record HIP events around every decode kernel launch."""
        _lib.check(_lib.lib().ldpc_ctx_profile(self._ctx, int(enable)))

    def kernel_time(self, reset=True):
        """(summed decode-kernel ms, launches) since the last reset."""
        ms, n = C.c_double(), C.c_int()
        _lib.check(_lib.lib().ldpc_ctx_kernel_time(self._ctx, C.byref(ms), C.byref(n), int(reset)))
        return ms.value, n.value

    KERNEL_NAMES = {0: "none", 1: "generic", 2: "windowed", 3: "windowed2_s16", 4: "windowed2_s32", 5: "coop", 6: "coop2", 7: "lds", 8: "coop3", 9: "ldsep", 10: "host", 11: "stairf"}

    @property
    def last_kernel(self):
        k = C.c_int()
        _lib.check(_lib.lib().ldpc_ctx_last_kernel(self._ctx, C.byref(k)))
        return self.KERNEL_NAMES.get(k.value, str(k.value))

    @property
    def last_et_stage(self):
        """First-stage iterations of the last decode's staged early
        termination on coop3 (0: one launch, or another kernel)."""
        k = C.c_int()
        _lib.check(_lib.lib().ldpc_ctx_last_et_stage(self._ctx, C.byref(k)))
        return k.value

    @property
    def last_skipped(self):
        """Name of the fastest kernel of this code that the last automatic
        selection could not use for its parameters (e.g. msg_max > 63 on the
        DVB-S2 fast paths), None when none was skipped."""
        k = C.c_int()
        _lib.check(_lib.lib().ldpc_ctx_last_skipped(self._ctx, C.byref(k)))
        return self.KERNEL_NAMES.get(k.value, str(k.value)) if k.value else None

    @property
    def stream(self):
        s = C.c_void_p()
        _lib.check(_lib.lib().ldpc_ctx_stream(self._ctx, C.byref(s)))
        return s.value

    # -- host buffers (synchronous)
    def decode_i8(self, llr, n_iter, params=None, out=None):
        llr = np.ascontiguousarray(llr, dtype=np.int8)
        B = llr.shape[0] if llr.ndim == 2 else 1
        assert llr.size == B * self.code.n, "llr must be [batch, N]"
        hard = out if out is not None else np.empty((B, self.code.n), dtype=np.uint8)
        p = params or _lib.default_params()
        _lib.check(_lib.lib().ldpc_decode_i8(self._ctx, llr.ctypes.data, hard.ctypes.data, B, n_iter, C.byref(p)))
        return hard

    def decode_f32(self, llr, n_iter, params=None, out=None):
        llr = np.ascontiguousarray(llr, dtype=np.float32)
        B = llr.shape[0] if llr.ndim == 2 else 1
        assert llr.size == B * self.code.n
        hard = out if out is not None else np.empty((B, self.code.n), dtype=np.uint8)
        p = params or _lib.default_params(algo=_lib.ALGO_MS)
        _lib.check(_lib.lib().ldpc_decode_f32(self._ctx, llr.ctypes.data, hard.ctypes.data, B, n_iter, C.byref(p)))
        return hard

    # -- host buffers, asynchronous (H2D -> decode -> D2H queued on `stream`)
    def decode_i8_host_async(self, llr, hard, n_iter, params=None, stream=None):
        """Queue the decode of host (preferably pinned_empty) arrays llr -> hard
        and return; hard is valid after synchronize().  One stream per context:
        use two contexts to keep two batches in flight."""
        assert llr.dtype == np.int8 and llr.flags.c_contiguous and hard.flags.c_contiguous
        B = llr.shape[0]
        assert llr.size == B * self.code.n and hard.size == B * self.code.n and hard.dtype == np.uint8
        p = params or _lib.default_params()
        self._on_stream(stream, lambda s: _lib.check(_lib.lib().ldpc_decode_i8_host_async(
            self._ctx, s, llr.ctypes.data, hard.ctypes.data, B, n_iter, C.byref(p))), self.device)
        # the queued copies read llr / write hard until synchronize(): keep the
        # arrays (and so a pinned_empty buffer's page-locked memory) alive --
        # every call's, since a second call may be queued before synchronize()
        self._pending.append((llr, hard))

    def synchronize(self):
        """Wait for this context's queued decode_i8_host_async calls."""
        _lib.check(_lib.lib().ldpc_ctx_synchronize(self._ctx))
        self._pending.clear()

    # -- device tensors (asynchronous on `stream`, default: torch current stream)
    @staticmethod
    def _ptr(t):
        return None if t is None else C.c_void_p(t.data_ptr())

    @staticmethod
    def _on_stream(stream, launch, device=None):
        """Run launch(hip_stream) on `stream`, default torch's current stream
        of `device`.  Handle 0 (torch's default stream) is HIP's null stream,
        which the C-ABI keeps as is (ordered with the legacy default stream)."""
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(device).cuda_stream
        return launch(C.c_void_p(stream) if stream else None)

    def decode_i8_device(self, llr, hard, n_iter, params=None, soft=None, iters_used=None, stream=None):
        B = llr.shape[0]
        assert llr.numel() == B * self.code.n and llr.is_contiguous()
        p = params or _lib.default_params()
        self._on_stream(stream, lambda s: _lib.check(_lib.lib().ldpc_decode_i8_async(
            self._ctx, s, self._ptr(llr), self._ptr(hard), self._ptr(soft), self._ptr(iters_used), B, n_iter,
            C.byref(p))), self.device)

    def decode_i8_nm_device(self, llr_nm, hard, n_iter, batch=None, params=None, soft=None, iters_used=None,
                            stream=None):
        """Node-major input llr_nm [N, ld] (codeword fastest; the reference's
        interleaved layout, CGPU_Decoder_MS_SIMD_v2::decode), `batch` <= ld
        codewords (default ld); hard / soft frame-major [batch, N]."""
        assert llr_nm.dim() == 2 and llr_nm.shape[0] == self.code.n and llr_nm.stride(1) == 1
        ld = llr_nm.stride(0)
        B = llr_nm.shape[1] if batch is None else batch
        assert B <= llr_nm.shape[1]
        p = params or _lib.default_params()
        self._on_stream(stream, lambda s: _lib.check(_lib.lib().ldpc_decode_i8_nm_async(
            self._ctx, s, self._ptr(llr_nm), ld, self._ptr(hard), self._ptr(soft), self._ptr(iters_used), B, n_iter,
            C.byref(p))), self.device)

    def decode_f32_device(self, llr, hard, n_iter, params=None, soft=None, iters_used=None, stream=None):
        B = llr.shape[0]
        assert llr.numel() == B * self.code.n and llr.is_contiguous()
        p = params or _lib.default_params(algo=_lib.ALGO_MS)
        self._on_stream(stream, lambda s: _lib.check(_lib.lib().ldpc_decode_f32_async(
            self._ctx, s, self._ptr(llr), self._ptr(hard), self._ptr(soft), self._ptr(iters_used), B, n_iter,
            C.byref(p))), self.device)

    def awgn_i8_device(self, llr, first_cw, seed, table, codeword=None, stream=None):
        t = np.ascontiguousarray(table, dtype=np.uint32)
        self._on_stream(stream, lambda s: _lib.check(_lib.lib().ldpc_awgn_i8_async(
            self._ctx, s, self._ptr(llr), llr.shape[0], first_cw, seed, t.ctypes.data, self._ptr(codeword))), self.device)

    def quantize_device(self, y, q, factor=8, sat_neg=-31, sat_pos=31, stream=None):
        """float -> int8 LLR on the device (CFastFixConversion::generate's rule:
        clamp(trunc(factor * y), sat_neg, sat_pos)); y float32, q int8, same numel."""
        assert y.is_contiguous() and q.is_contiguous() and y.numel() == q.numel()
        self._on_stream(stream, lambda s: _lib.check(_lib.lib().ldpc_quantize_f32_i8_async(
            self._ctx, s, self._ptr(y), self._ptr(q), y.numel(), factor, sat_neg, sat_pos)), self.device)

    def quantize(self, y, factor=8, sat_neg=-31, sat_pos=31):
        """Host arrays: float32 -> int8 through the device (synchronous)."""
        y = np.ascontiguousarray(y, dtype=np.float32)
        q = np.empty(y.shape, dtype=np.int8)
        _lib.check(_lib.lib().ldpc_quantize_f32_i8(self._ctx, y.ctypes.data, q.ctypes.data, y.size, factor, sat_neg,
                                                   sat_pos))
        return q

    def decode_count_device(self, llr, hard, n_iter, k, counts, ref=None, params=None, soft=None, iters_used=None,
                            stream=None):
        """decode_*_device + count_errors_device in one call (float or int8 by
        llr's dtype): counts[0] += bit errors over the first k bits vs ref
        (None: the all-zero codeword), counts[1] += frame errors; fused into
        the edge-parallel float kernel's epilogue."""
        import torch
        B = llr.shape[0]
        assert llr.numel() == B * self.code.n and llr.is_contiguous()
        f32 = llr.dtype == torch.float32
        p = params or (_lib.default_params(algo=_lib.ALGO_MS) if f32 else _lib.default_params())
        fn = _lib.lib().ldpc_decode_f32_count_async if f32 else _lib.lib().ldpc_decode_i8_count_async
        self._on_stream(stream, lambda s: _lib.check(fn(
            self._ctx, s, self._ptr(llr), self._ptr(hard), self._ptr(soft), self._ptr(iters_used), B, n_iter,
            C.byref(p), int(k), self._ptr(ref), self._ptr(counts))), self.device)

    def count_errors_device(self, hard, k, counts, ref=None, stream=None):
        self._on_stream(stream, lambda s: _lib.check(_lib.lib().ldpc_count_errors_async(
            self._ctx, s, self._ptr(hard), hard.shape[0], k, self._ptr(ref), self._ptr(counts))), self.device)

    def close(self):
        if getattr(self, "_ctx", None) is not None and _lib._lib is not None:
            _lib._lib.ldpc_ctx_destroy(self._ctx)   # waits for the context's stream
            self._ctx = None
        getattr(self, "_pending", []).clear()

    def __del__(self):
        self.close()


class MixedDecoder:
    """Mixed-rate batches (codes of equal N, e.g. the DVB-S2 normal-frame
    rates): per-code contexts decoding their codewords concurrently."""

    def __init__(self, codes, device=0, max_batch=4096):
        self.codes = [c if isinstance(c, Code) else Code(c) for c in codes]
        arr = (C.c_void_p * len(self.codes))(*[c.handle for c in self.codes])
        h = C.c_void_p()
        _lib.check(_lib.lib().ldpc_mixed_create(arr, len(self.codes), device, max_batch, C.byref(h)))
        self._mx = h
        self.n = self.codes[0].n
        self.device = device

    def decode_i8_device(self, llr, hard, code_id, n_iter, params=None, iters_used=None, stream=None):
        """llr/hard: device tensors [B, N]; code_id: host int array [B]."""
        ids = np.ascontiguousarray(code_id, dtype=np.int32)
        p = params or _lib.default_params()
        Decoder._on_stream(stream, lambda s: _lib.check(_lib.lib().ldpc_decode_i8_mixed_async(
            self._mx, s, Decoder._ptr(llr), Decoder._ptr(hard), Decoder._ptr(iters_used), ids.ctypes.data,
            ids.size, n_iter, C.byref(p))), self.device)

    def last_kernels(self):
        """Kernel family each code's sub-batch ran in the last decode (names as
        Decoder.last_kernel; "none" for a code without codewords so far)."""
        out = []
        for c in range(len(self.codes)):
            k = C.c_int()
            _lib.check(_lib.lib().ldpc_mixed_last_kernel(self._mx, c, C.byref(k)))
            out.append(Decoder.KERNEL_NAMES.get(k.value, str(k.value)))
        return out

    def last_et_stages(self):
        """Per code: first-stage iterations of its last staged early
        termination (Decoder.last_et_stage; 0 = one launch)."""
        out = []
        for c in range(len(self.codes)):
            k = C.c_int()
            _lib.check(_lib.lib().ldpc_mixed_last_et_stage(self._mx, c, C.byref(k)))
            out.append(k.value)
        return out

    def profile(self, enable=True):
        """Record each code's decode-kernel launches with HIP events."""
        _lib.check(_lib.lib().ldpc_mixed_profile(self._mx, int(bool(enable))))

    def kernel_time(self, reset=True):
        """[(total_ms, launches)] per code since the last reset (profile() on)."""
        out = []
        for c in range(len(self.codes)):
            ms, n = C.c_double(), C.c_int()
            _lib.check(_lib.lib().ldpc_mixed_kernel_time(self._mx, c, C.byref(ms), C.byref(n), int(reset)))
            out.append((ms.value, n.value))
        return out

    def close(self):
        if getattr(self, "_mx", None) is not None and _lib._lib is not None:
            _lib._lib.ldpc_mixed_destroy(self._mx)
            self._mx = None

    def __del__(self):
        self.close()


# ---------------------------------------------------------------------------
# Reference-shaped mirror (CDecoder hierarchy + CreateDecoder factory)

@dataclass
class param_decoder:
    """code/x86/main_p.cpp:133-141 defaults."""
    nb_iters: int = 30
    nms_factor_fixed: int = 29
    nms_factor_float: float = 0.75
    oms_offset_fixed: int = 1
    oms_offset_float: float = 0.15


class CDecoder:
    """code/x86/CDecoder/template/CDecoder.h:28-40."""

    def __init__(self, code, nb_frames=16, device=0):
        self._dec = Decoder(code, device=device, max_batch=nb_frames)
        self.nb_frames = nb_frames
        self.sigB = 0.0
        self.nb_iters = 0
        self._p = _lib.default_params()

    def setSigmaChannel(self, sigB):
        self.sigB = float(sigB)

    def setNumberOfIterations(self, value):
        self.nb_iters = int(value)

    def decode(self, var_nodes, Rprime_fix, nombre_iterations):
        """decode(char llr[], char hard[], int it): int8 in, 0/1 out, in place.
        A float llr array selects the float decoder (the reference's
        fixed-point decoders ignore that overload, CDecoder_fixed_SSE.cpp:35-40;
        here it runs the float layered min-sum)."""
        n = self._dec.code.n
        arr = np.asarray(var_nodes)
        frames = arr.size // n
        out = np.asarray(Rprime_fix).reshape(frames, n) if isinstance(Rprime_fix, np.ndarray) else None
        if arr.dtype == np.float32 or arr.dtype == np.float64:
            res = self._dec.decode_f32(arr.reshape(frames, n), nombre_iterations, self._float_params())
        else:
            res = self._dec.decode_i8(arr.reshape(frames, n), nombre_iterations, self._p)
        if out is not None:
            out[...] = res
        return res

    def _float_params(self):
        return _lib.default_params(algo=_lib.ALGO_MS)


class CDecoder_fixed(CDecoder):
    """code/x86/CDecoder/template/CDecoder_fixed.h:30-44."""

    def setVarRange(self, vmin, vmax):
        self._p.var_min, self._p.var_max = int(vmin), int(vmax)

    def setMsgRange(self, mmin, mmax):
        self._p.msg_min, self._p.msg_max = int(mmin), int(mmax)


class CDecoder_OMS_fixed_MI355X(CDecoder_fixed):
    """Offset min-sum (code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.h)."""

    def __init__(self, code, nb_frames=16, device=0):
        super().__init__(code, nb_frames, device)
        self._p.algo = _lib.ALGO_OMS
        self._offset_set = False

    def setOffset(self, offset):
        # single assignment, as CDecoder_OMS_fixed_SSE::setOffset (:104-112)
        if self._offset_set:
            raise _lib.LdpcError(_lib.LDPC_EINVAL, "Offset value was already configured (%d)" % self._p.offset)
        self._p.offset = int(offset)
        self._offset_set = True


class CDecoder_NMS_fixed_MI355X(CDecoder_fixed):
    """Normalised min-sum (code/x86/CDecoder/NMS/CDecoder_NMS_fixed_SSE.h)."""

    def __init__(self, code, nb_frames=16, device=0):
        super().__init__(code, nb_frames, device)
        self._p.algo = _lib.ALGO_NMS

    def setFactor(self, factor):
        self._p.factor = int(factor)


def CreateDecoder(type, arch, format, p_decoder, vMin, vMax, mMin, mMax, code="576x288", nb_frames=16, device=0):
    """code/x86/CDecoder/DecoderLibrary.h:44-134 (arch "mi355x" instead of "sse")."""
    if arch not in ("mi355x", "gpu", "sse"):
        raise _lib.LdpcError(_lib.LDPC_EUNSUPPORTED, "decoder unavailable: arch %s" % arch)
    if format != "fixed":
        raise _lib.LdpcError(_lib.LDPC_EUNSUPPORTED, "decoder unavailable: format %s" % format)
    if type == "OMS":
        d = CDecoder_OMS_fixed_MI355X(code, nb_frames, device)
        d.setOffset(p_decoder.oms_offset_fixed)
    elif type == "NMS":
        d = CDecoder_NMS_fixed_MI355X(code, nb_frames, device)
        d.setFactor(p_decoder.nms_factor_fixed)
    else:
        raise _lib.LdpcError(_lib.LDPC_EUNSUPPORTED, "Requested LDPC decoder does not exist (%s:%s)" % (arch, type))
    d.setVarRange(vMin, vMax)
    d.setMsgRange(mMin, mMax)
    return d

"""ctypes binding of libavse.so (include/avse.h).

`import torch` must happen before libavse.so is loaded: both link libamdhip64.so.7, so loading
torch first makes libavse share torch's HIP runtime (one set of streams / allocations).

There is no fallback: if libavse.so is missing or fails to load, every entry point raises.
"""
import contextlib
import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

# AVSE_LIBRARY selects another build of the same ABI, e.g. the checked build (csrc/Makefile DEBUG=1 -> libavse_debug.so)
LIB_PATH = os.environ.get("AVSE_LIBRARY") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libavse.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "avse.h")

ABI_VERSION = 3
AVSE_F32 = 0
AVSE_BF16 = 1
AVSE_F32_SPLIT = 2
AVSE_PAD_REFLECT = 0
AVSE_PAD_CONSTANT = 1
AVSE_ERR_RANGE = 6
AVSE_RANGE_RECOMPUTE, AVSE_RANGE_ERROR = 0, 1
# range-guard bits (include/avse.h avse_forward_checked): bit i = plan layer i, 24 / 25 the split audio / video inputs
LAYER_NAMES = ("a_conv1", "a_conv2", "a_conv3", "a_conv4", "a_conv5", "v_conv1", "v_conv2", "v_conv3", "v_conv4",
               "v_conv5", "v_conv6", "enc_dense", "dec_dense1", "dec_dense2", "d_deconv1", "d_deconv2", "d_deconv3",
               "d_deconv4", "d_deconv5", "d_deconv6")


def range_bit_names(bits):
    """The layers / inputs a range-guard word names."""
    names = [n for i, n in enumerate(LAYER_NAMES) if bits >> i & 1]
    return names + [n for b, n in ((24, "audio input"), (25, "video input")) if bits >> b & 1]
AVSE_NUM_STAGES = 22
STAGE_NAMES = ("video_prep", "audio_prep", "a_conv1", "a_conv2", "a_conv3", "a_conv4", "a_conv5",
               "v_conv1", "v_conv2", "v_conv3", "v_conv4", "v_conv5", "v_conv6", "enc_dense", "dec_dense1",
               "dec_dense2", "d_deconv1", "d_deconv2", "d_deconv3", "d_deconv4", "d_deconv5", "d_deconv6")

_c_void_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int
_flt = ctypes.c_float

# name -> (restype, argtypes); every function declared in include/avse.h
SIGNATURES = {
    "avse_abi_version": (_int, []),
    "avse_build_flags": (_int, []),
    "avse_last_error": (ctypes.c_char_p, []),
    "avse_ctx_create": (_int, [_int, ctypes.POINTER(_c_void_p)]),
    "avse_ctx_destroy": (None, [_c_void_p]),
    "avse_ctx_reserve": (_int, [_c_void_p, _i64, _int]),
    "avse_ctx_reserve_weights": (_int, [_c_void_p, _c_void_p, _i64]),
    "avse_ctx_set_option": (_int, [_c_void_p, ctypes.c_char_p, _int]),
    "avse_ctx_get_option": (_int, [_c_void_p, ctypes.c_char_p, ctypes.POINTER(_int)]),
    "avse_spectrogram": (_int, [_c_void_p, _c_void_p, _i64, _i64, _int, _int, _int, _int, _flt, _flt, _flt, _flt,
                                _int, _int, _c_void_p, _c_void_p, _c_void_p]),
    "avse_istft": (_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _int, _int, _int, _int, _int, _int, _int, _flt, _flt,
                          _c_void_p, _c_void_p]),
    "avse_weights_blob_floats": (_i64, []),
    "avse_weights_load": (_int, [_c_void_p, _c_void_p, _i64, _int, ctypes.POINTER(_c_void_p)]),
    "avse_weights_blob_floats_shape": (_i64, [_int, _int]),
    "avse_weights_load_shape": (_int, [_c_void_p, _c_void_p, _i64, _int, _int, _int, ctypes.POINTER(_c_void_p)]),
    "avse_weights_shape": (_int, [_c_void_p, ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "avse_weights_destroy": (None, [_c_void_p]),
    "avse_forward": (_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p,
                            _c_void_p]),
    "avse_video_normalize": (_int, [_c_void_p, _c_void_p, _i64, _int, _int, _int, _c_void_p, _c_void_p, _c_void_p]),
    "avse_mse": (_int, [_c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p]),
    "avse_forward_checked": (_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p,
                                    _c_void_p, _int, ctypes.POINTER(ctypes.c_uint32)]),
    "avse_range_status": (_int, [_c_void_p, _c_void_p, ctypes.POINTER(ctypes.c_uint32)]),
    "avse_range_snapshot": (_int, [_c_void_p, _c_void_p, _c_void_p]),
    "avse_weights_act_exponents": (_int, [_c_void_p, ctypes.POINTER(_int), _int]),
    "avse_forward_profile": (_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64,
                                    _c_void_p, _c_void_p, ctypes.POINTER(_flt)]),
    "avse_debug_scratch": (_int, [_c_void_p, _i64, _int, ctypes.POINTER(_c_void_p), ctypes.POINTER(_i64)]),
    "avse_trainer_create": (_int, [_c_void_p, _c_void_p, _i64, _i64, ctypes.POINTER(_c_void_p)]),
    "avse_trainer_create_shape": (_int, [_c_void_p, _c_void_p, _i64, _i64, _int, _int, ctypes.POINTER(_c_void_p)]),
    "avse_trainer_destroy": (None, [_c_void_p]),
    "avse_trainer_step": (_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _flt, _flt,
                                 ctypes.c_uint32, _int, _c_void_p, _c_void_p]),
    "avse_trainer_read": (_int, [_c_void_p, _int, _c_void_p, _i64]),
    "avse_trainer_iterations": (_int, [_c_void_p, ctypes.POINTER(_i64)]),
}
AVSE_TRAIN_PARAMS, AVSE_TRAIN_GRADS, AVSE_TRAIN_ADAM_M, AVSE_TRAIN_ADAM_V = 0, 1, 2, 3
AVSE_TRAIN_GRADS_ONLY = 1


def source_digest():
    """sha256 (first 16 hex digits) of the sources libavse.so is built from: csrc/*.hip, csrc/*.h, csrc/Makefile and
    include/avse.h.  Profiles record it (tools/pmc_summary.py) so that bench.py attaches rocprof counters only to the
    tree they were measured on — the GPU box has no .git to name a commit."""
    import glob
    import hashlib
    pkg = os.path.dirname(os.path.abspath(__file__))
    files = sorted(glob.glob(os.path.join(pkg, "csrc", "*.hip")) + glob.glob(os.path.join(pkg, "csrc", "*.h")) +
                   [os.path.join(pkg, "csrc", "Makefile"), HEADER_PATH])
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


class AvseError(RuntimeError):
    """A libavse call returned a non-zero status."""


_lock = threading.Lock()
_lib = None


def load():
    """Load libavse.so (once) and declare every signature.  Raises if it is missing."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise AvseError(
                    f"{LIB_PATH} is not built: run `make -C audio-visual-speech-enhancement_amd/csrc` "
                    "(or __graft_entry__.build()); there is no CPU fallback")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            if lib.avse_abi_version() != ABI_VERSION:
                raise AvseError(f"{LIB_PATH} implements ABI {lib.avse_abi_version()}, this binding ABI {ABI_VERSION}: rebuild it")
            _lib = lib
    return _lib


class RangeError(AvseError):
    """avse_forward_checked(AVSE_RANGE_ERROR): an AVSE_F32_SPLIT activation left the f16 pair range."""


def check(rc, what):
    if rc != 0:
        msg = load().avse_last_error().decode(errors="replace")
        raise (RangeError if rc == AVSE_ERR_RANGE else AvseError)(f"{what} failed (status {rc}): {msg}")


class Context:
    """One libavse context per device (avse_ctx_create)."""

    def __init__(self, device_index):
        self.device_index = device_index
        self._cdll = load()   # held for __del__: module globals may be torn down first at interpreter exit
        self.handle = _c_void_p()
        self._set_aside = 0
        check(load().avse_ctx_create(device_index, ctypes.byref(self.handle)), "avse_ctx_create")

    def _read_range(self, stream):
        bits = ctypes.c_uint32()
        check(load().avse_range_status(self.handle, stream if stream is not None else stream_handle(self.device_index),
                                       ctypes.byref(bits)), "avse_range_status")
        return bits.value

    def range_status(self, stream=None):
        """avse_range_status: the range-guard bits raised by unchecked split forwards since the last call (waits for
        `stream`, default torch's current stream on this device, and clears them), plus any bits set_aside_range()
        took out of the device word since then.

        The guard word is one per context (include/avse.h): forwards of one context on several streams or threads OR
        into the same word, so a reader cannot tell which of them raised a bit.  Give each concurrent pipeline its own
        context (avse_ctx_create) when that matters."""
        bits = self._read_range(stream) | self._set_aside
        self._set_aside = 0
        return bits

    def set_aside_range(self, stream=None):
        """Start a pipeline with a clean device guard word WITHOUT discarding what earlier forwards raised: their bits
        move to the host side and the next range_status() still returns them (pipeline.Enhancer, bench.py)."""
        self._set_aside |= self._read_range(stream)

    def reserve(self, max_clips, dtype):
        check(load().avse_ctx_reserve(self.handle, int(max_clips), int(dtype)), "avse_ctx_reserve")

    def reserve_for(self, weights, max_clips):
        """avse_ctx_reserve_weights: scratch for `weights`' network shape and dtype (ops.DeviceWeights)."""
        check(load().avse_ctx_reserve_weights(self.handle, weights.handle, int(max_clips)), "avse_ctx_reserve_weights")

    def set_option(self, name, value):
        """avse_ctx_set_option: a kernel-path switch (include/avse.h), e.g. "no_gemm"."""
        check(load().avse_ctx_set_option(self.handle, name.encode(), int(value)), f"avse_ctx_set_option({name})")

    def get_option(self, name):
        v = _int()
        check(load().avse_ctx_get_option(self.handle, name.encode(), ctypes.byref(v)), f"avse_ctx_get_option({name})")
        return v.value

    @contextlib.contextmanager
    def options(self, **switches):
        """Temporarily set kernel-path switches: `with ctx.options(no_gemm=1): ...`."""
        old = {k: self.get_option(k) for k in switches}
        try:
            for k, v in switches.items():
                self.set_option(k, v)
            yield self
        finally:
            for k, v in old.items():
                self.set_option(k, v)

    def __del__(self):
        h, lib = getattr(self, "handle", None), getattr(self, "_cdll", None)
        if h is not None and h.value and lib is not None:
            lib.avse_ctx_destroy(h)
            self.handle = None


_ctx = {}


def context(device=None):
    if not torch.cuda.is_available():
        raise AvseError("libavse needs a ROCm GPU (torch.cuda.is_available() is False); there is no CPU fallback")
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    with _lock:
        c = _ctx.get(idx)
    if c is None:
        c = Context(idx)
        with _lock:
            _ctx[idx] = c
    return c


def stream_handle(device=None):
    return _c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return _c_void_p(t.data_ptr()) if t is not None else _c_void_p(None)

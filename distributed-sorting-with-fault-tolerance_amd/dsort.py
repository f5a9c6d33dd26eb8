"""ctypes binding of libdsort (include/dsort.h) for tests, the bench and __graft_entry__.

The product is the C ABI in lib/libdsort.so (HIP kernels for gfx950); this module only loads it
and converts arguments.  There is no fallback: if the library is missing or no gfx950 device is
present, the calls raise.  torch is imported BEFORE the library so that libdsort binds to the HIP
runtime torch already loaded (same soname libamdhip64.so.7): device memory from torch tensors and
the library's kernels then live in one runtime.
"""
import contextlib
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# DSORT_LIB: an alternative build of the same library (A/B experiments of compile-time variants)
LIB_PATH = os.environ.get("DSORT_LIB") or os.path.join(HERE, "lib", "libdsort.so")

try:  # shared HIP runtime (see module docstring); absence of torch is fine on the CPU box
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    torch = None

DSORT_OK = 0
DSORT_ECOMM = -4
DSORT_ETIMEOUT = -6
ERRORS = {-1: "EINVAL", -2: "ENOMEM", -3: "EHIP", -4: "ECOMM", -5: "ENODEV", -6: "ETIMEOUT", -7: "ESTAGE"}

# every symbol include/dsort.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "dsort_init", "dsort_finalize", "dsort_last_error", "dsort_version", "dsort_get_stats",
    "dsort_synchronize", "dsort_set_option", "dsort_get_option", "dsort_sort_stages", "dsort_sample_sort_stages", "dsort_sort_i32", "dsort_sort_i64", "dsort_sort_dev_i32",
    "dsort_sort_dev_i64", "dsort_sort_dev_copy_i32", "dsort_sort_dev_copy_i64",
    "dsort_merge_i32", "dsort_merge_i64", "dsort_merge_dev_i32", "dsort_merge_dev_i64",
    "dsort_comm_unique_id", "dsort_comm_init", "dsort_comm_init_transport", "dsort_comm_abort",
    "dsort_comm_destroy", "dsort_comm_deadline_ms",
    "dsort_sample_sort_dev_i32", "dsort_sample_sort_dev_i64", "dsort_sample_merge_dev_i32",
    "dsort_sample_merge_dev_i64", "dsort_plan_splitters_i32",
    "dsort_plan_splitters_i64", "dsort_plan_cuts_i32", "dsort_plan_cuts_i64",
    "dsort_plan_sample_positions", "dsort_gen_uniform_i32", "dsort_gen_uniform_i64",
    "dsort_gen_zipf_i64", "dsort_fingerprint_i32", "dsort_fingerprint_i64",
    "dsort_count_descents_i32", "dsort_count_descents_i64", "dsort_dev_alloc", "dsort_dev_free",
    "dsort_copy_h2d", "dsort_copy_d2h", "dsort_copy_d2d", "dsort_host_register",
    "dsort_host_unregister", "dsort_write_text_i32", "dsort_format_text_dev_i32",
    "dsort_parse_text_dev_i32", "dsort_parse_text_i32", "dsort_format_text_i32",
]


# dsort_set_option / dsort_get_option (include/dsort.h)
OPTIONS = {"buckets": 1, "bucket_keys": 2, "bucket_oversample": 3,
           "max_fanin_log2": 5, "kill_after_stage": 6, "kill_in_exchange": 7,
           "comm_timeout_ms": 8,
           "sub_keys": 9, "sub_oversample": 10, "sub_gather": 11, "test_hold_exchange": 12,
           "test_fail_exchange": 13, "stage_timing": 14, "test_tile_cap": 15,
           "test_wave_fence": 16}


class DsortError(RuntimeError):
    pass


class Stats(ctypes.Structure):
    _fields_ = [("block_sort_ms", ctypes.c_double), ("merge_ms", ctypes.c_double),
                ("exchange_ms", ctypes.c_double), ("final_merge_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double), ("merge_kernel_ms", ctypes.c_double),
                ("merge_kernel_launches", ctypes.c_int), ("merge_passes", ctypes.c_int),
                ("tile_keys", ctypes.c_int), ("keys_in", ctypes.c_size_t),
                ("keys_out", ctypes.c_size_t), ("alltoall_ms", ctypes.c_double),
                ("keys_sent", ctypes.c_size_t), ("tile_sort_kernel_ms", ctypes.c_double),
                ("partition_ms", ctypes.c_double), ("tile_sort_keys", ctypes.c_size_t),
                ("bucket_hist_ms", ctypes.c_double), ("bucket_scatter_ms", ctypes.c_double),
                ("sub_partition_ms", ctypes.c_double), ("sub_split_subbuckets", ctypes.c_int),
                ("sub_scatter_fallback", ctypes.c_int), ("exchange_path", ctypes.c_int),
                ("first_level_map", ctypes.c_int),
                ("fence_ranges", ctypes.c_int),  # ABI 6
                ("deferred_frees", ctypes.c_int), ("pending_frees", ctypes.c_int)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_size_t)
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t),
                                ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                ctypes.POINTER(ctypes.c_size_t))


class Transport(ctypes.Structure):
    """dsort_transport: the sample sort's exchanges through host callbacks (dsort.h)."""
    _fields_ = [("user", ctypes.c_void_p), ("allgather", ALLGATHER_FN), ("alltoallv", ALLTOALLV_FN)]


def torch_dist_transport(world, pg=None, deadline_fn=None):
    """A dsort_transport over a torch.distributed process group (gloo: CPU tensors; the default
    group unless `pg` is given).  For ranks that share a GPU, where RCCL refuses to build a
    communicator, and for the survivors' group after a fault (ftsort.py).

    Every wait is bounded by the exchange deadline: `deadline_fn()` gives the milliseconds left
    (-1 = none).  Context.comm_init_transport sets it to dsort_comm_deadline_ms, so a collective
    whose peer never arrives returns DSORT_ETIMEOUT (-6) at the sort's DSORT_OPT_COMM_TIMEOUT_MS
    instead of blocking until gloo's own timeout (dsort.h, ABI 5).

    A timed-out gloo operation stays queued on the group, so a later collective on it could pair
    with a slow peer's stale one (a status gate and a key count are both 8 bytes).  After the first
    timeout the transport is therefore POISONED: every later callback fails at once (the sort
    returns DSORT_ECOMM) and the group must be rebuilt, as ftsort.py does for its survivors."""
    import datetime

    import torch.distributed as dist

    def _wait(work):
        fn = t.deadline_fn
        ms = fn() if fn is not None else -1
        if ms is None or ms < 0:
            work.wait()
            return 0
        try:
            work.wait(timeout=datetime.timedelta(milliseconds=max(int(ms), 1)))
        except RuntimeError as e:
            if "timed out" in str(e).lower():
                print("dsort host transport: no answer before the exchange deadline", flush=True)
                t.poisoned = "a collective timed out at the exchange deadline"
                return DSORT_ETIMEOUT
            raise
        return 0

    def _allgather(user, send, recv, nbytes):
        if t.poisoned:
            return DSORT_ECOMM
        try:
            mine = torch.frombuffer(bytearray(ctypes.string_at(send, nbytes)), dtype=torch.uint8) \
                if nbytes else torch.empty(0, dtype=torch.uint8)
            outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(world)]
            if pg is None:
                work = dist.all_gather(outs, mine, async_op=True)
            else:
                work = pg.allgather([outs], [mine])
            rc = _wait(work)
            if rc:
                return rc
            if nbytes:
                whole = torch.cat(outs).numpy()
                ctypes.memmove(recv, whole.ctypes.data, whole.nbytes)
            return 0
        except Exception as e:  # pragma: no cover - reported through the C error path
            print("dsort host transport allgather:", e, flush=True)
            return 1

    def _alltoallv(user, send, sc, sd, recv, rc, rd):
        if t.poisoned:
            return DSORT_ECOMM
        try:
            scounts = [int(sc[i]) for i in range(world)]
            rcounts = [int(rc[i]) for i in range(world)]
            chunks = b"".join(ctypes.string_at(send + int(sd[i]), scounts[i]) if scounts[i] else b""
                              for i in range(world))
            inp = torch.frombuffer(bytearray(chunks), dtype=torch.uint8) if chunks else torch.empty(0, dtype=torch.uint8)
            out = torch.empty(sum(rcounts), dtype=torch.uint8)
            if pg is None:
                work = dist.all_to_all_single(out, inp, output_split_sizes=rcounts, input_split_sizes=scounts,
                                              async_op=True)
            else:
                work = pg.alltoall_base(out, inp, rcounts, scounts)
            r = _wait(work)
            if r:
                return r
            o = out.numpy()
            off = 0
            for i in range(world):
                if rcounts[i]:
                    ctypes.memmove(recv + int(rd[i]), o.ctypes.data + off, rcounts[i])
                off += rcounts[i]
            return 0
        except Exception as e:  # pragma: no cover
            print("dsort host transport alltoallv:", e, flush=True)
            return 1

    t = Transport(None, ALLGATHER_FN(_allgather), ALLTOALLV_FN(_alltoallv))
    t._keep = (_allgather, _alltoallv)  # the C side holds raw function pointers
    t.deadline_fn = deadline_fn
    t.poisoned = None  # (set by the first timeout: the group must be rebuilt)
    return t


_lib = None
P = ctypes.c_void_p
SZ = ctypes.c_size_t
U64 = ctypes.c_uint64
I32 = ctypes.c_int32


def load():
    """Load lib/libdsort.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DsortError(f"{LIB_PATH} missing: build it with `make -C {HERE}` (no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    sig = {
        "dsort_init": (ctypes.c_int, [ctypes.POINTER(P), ctypes.c_int]),
        "dsort_finalize": (ctypes.c_int, [P]),
        "dsort_last_error": (ctypes.c_char_p, [P]),
        "dsort_version": (ctypes.c_char_p, []),
        "dsort_get_stats": (ctypes.c_int, [P, ctypes.POINTER(Stats)]),
        "dsort_synchronize": (ctypes.c_int, [P]),
        "dsort_set_option": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int64]),
        "dsort_get_option": (ctypes.c_int, [P, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]),
        "dsort_sort_stages": (ctypes.c_int, [P, SZ, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
        "dsort_sample_sort_stages": (ctypes.c_int, [P, SZ, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    ctypes.POINTER(ctypes.c_int)]),
        "dsort_sort_i32": (ctypes.c_int, [P, P, SZ]),
        "dsort_sort_i64": (ctypes.c_int, [P, P, SZ]),
        "dsort_sort_dev_i32": (ctypes.c_int, [P, P, SZ, P]),
        "dsort_sort_dev_i64": (ctypes.c_int, [P, P, SZ, P]),
        "dsort_sort_dev_copy_i32": (ctypes.c_int, [P, P, P, SZ, P]),
        "dsort_sort_dev_copy_i64": (ctypes.c_int, [P, P, P, SZ, P]),
        "dsort_merge_i32": (ctypes.c_int, [P, P, P, ctypes.c_int, P]),
        "dsort_merge_i64": (ctypes.c_int, [P, P, P, ctypes.c_int, P]),
        "dsort_merge_dev_i32": (ctypes.c_int, [P, P, P, ctypes.c_int, P, P]),
        "dsort_merge_dev_i64": (ctypes.c_int, [P, P, P, ctypes.c_int, P, P]),
        "dsort_comm_unique_id": (ctypes.c_int, [P]),
        "dsort_comm_init": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, P]),
        "dsort_comm_init_transport": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(Transport)]),
        "dsort_comm_abort": (ctypes.c_int, [P]),
        "dsort_comm_deadline_ms": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_int64)]),
        "dsort_comm_destroy": (ctypes.c_int, [P]),
        "dsort_sample_sort_dev_i32": (ctypes.c_int, [P, P, SZ, ctypes.POINTER(P), ctypes.POINTER(SZ), P]),
        "dsort_sample_sort_dev_i64": (ctypes.c_int, [P, P, SZ, ctypes.POINTER(P), ctypes.POINTER(SZ), P]),
        "dsort_sample_merge_dev_i32": (ctypes.c_int, [P, P, SZ, ctypes.POINTER(P), ctypes.POINTER(SZ), P]),
        "dsort_sample_merge_dev_i64": (ctypes.c_int, [P, P, SZ, ctypes.POINTER(P), ctypes.POINTER(SZ), P]),
        "dsort_plan_splitters_i32": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, P, P, P, P, P]),
        "dsort_plan_splitters_i64": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, P, P, P, P, P]),
        "dsort_plan_cuts_i32": (ctypes.c_int, [P, SZ, ctypes.c_int, ctypes.c_int, P, P, P, P]),
        "dsort_plan_cuts_i64": (ctypes.c_int, [P, SZ, ctypes.c_int, ctypes.c_int, P, P, P, P]),
        "dsort_plan_sample_positions": (ctypes.c_int, [SZ, ctypes.c_int, P]),
        "dsort_gen_uniform_i32": (ctypes.c_int, [P, P, SZ, U64, U64, P]),
        "dsort_gen_uniform_i64": (ctypes.c_int, [P, P, SZ, U64, U64, P]),
        "dsort_gen_zipf_i64": (ctypes.c_int, [P, P, SZ, U64, U64, P]),
        "dsort_fingerprint_i32": (ctypes.c_int, [P, P, SZ, ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        "dsort_fingerprint_i64": (ctypes.c_int, [P, P, SZ, ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        "dsort_count_descents_i32": (ctypes.c_int, [P, P, SZ, ctypes.POINTER(U64)]),
        "dsort_count_descents_i64": (ctypes.c_int, [P, P, SZ, ctypes.POINTER(U64)]),
        "dsort_dev_alloc": (ctypes.c_int, [P, ctypes.POINTER(P), SZ]),
        "dsort_dev_free": (ctypes.c_int, [P, P]),
        "dsort_copy_h2d": (ctypes.c_int, [P, P, P, SZ]),
        "dsort_copy_d2h": (ctypes.c_int, [P, P, P, SZ]),
        "dsort_copy_d2d": (ctypes.c_int, [P, P, P, SZ]),
        "dsort_host_register": (ctypes.c_int, [P, P, SZ]),
        "dsort_host_unregister": (ctypes.c_int, [P, P]),
        "dsort_write_text_i32": (ctypes.c_int, [ctypes.c_char_p, P, SZ]),
        "dsort_format_text_dev_i32": (ctypes.c_int, [P, P, SZ, P, SZ, ctypes.POINTER(SZ), P]),
        "dsort_parse_text_dev_i32": (ctypes.c_int, [P, P, SZ, P, SZ, ctypes.POINTER(SZ), P]),
        "dsort_parse_text_i32": (ctypes.c_int, [P, ctypes.c_char_p, SZ, P, SZ, ctypes.POINTER(SZ)]),
        "dsort_format_text_i32": (ctypes.c_int, [P, P, SZ, P, SZ, ctypes.POINTER(SZ)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def _ptr(a):
    return a.ctypes.data if isinstance(a, np.ndarray) else a


def _sfx(dtype):
    dt = np.dtype(dtype)
    if dt == np.int32:
        return "i32"
    if dt == np.int64:
        return "i64"
    raise DsortError(f"unsupported key type {dt} (int32 / int64)")


# ----------------------------------------------------------------- host-only planning helpers
def plan_sample_positions(n, s):
    lib = load()
    idx = np.zeros(s, np.uint64)
    _check(None, lib.dsort_plan_sample_positions(n, s, _ptr(idx)))
    return idx


def plan_splitters(samples, idx, nranks):
    """samples: (nranks*s,) keys, per-rank sorted blocks; returns (val, rank, index) arrays."""
    lib = load()
    samples = np.ascontiguousarray(samples)
    s = samples.size // nranks
    sv = np.zeros(max(nranks - 1, 1), samples.dtype)
    sr = np.zeros(max(nranks - 1, 1), np.int32)
    si = np.zeros(max(nranks - 1, 1), np.uint64)
    f = getattr(lib, f"dsort_plan_splitters_{_sfx(samples.dtype)}")
    _check(None, f(nranks, s, _ptr(samples), _ptr(np.ascontiguousarray(idx, np.uint64)),
                   _ptr(sv), _ptr(sr), _ptr(si)))
    return sv[:nranks - 1], sr[:nranks - 1], si[:nranks - 1]


def plan_cuts(sorted_keys, my_rank, nranks, sv, sr, si):
    lib = load()
    sorted_keys = np.ascontiguousarray(sorted_keys)
    cuts = np.zeros(nranks + 1, np.uint64)
    f = getattr(lib, f"dsort_plan_cuts_{_sfx(sorted_keys.dtype)}")
    sv = np.ascontiguousarray(sv, sorted_keys.dtype)
    sr = np.ascontiguousarray(sr, np.int32)
    si = np.ascontiguousarray(si, np.uint64)
    _check(None, f(_ptr(sorted_keys), sorted_keys.size, my_rank, nranks, _ptr(sv), _ptr(sr),
                   _ptr(si), _ptr(cuts)))
    return cuts


def write_text_i32(path, keys):
    lib = load()
    keys = np.ascontiguousarray(keys, np.int32)
    _check(None, lib.dsort_write_text_i32(os.fsencode(path), _ptr(keys), keys.size))


def _check(ctx, rc):
    if rc != DSORT_OK:
        msg = load().dsort_last_error(ctx).decode() if ctx else ""
        err = DsortError(f"libdsort error {rc} ({ERRORS.get(rc, '?')}): {msg}")
        err.rc = rc
        raise err
    return rc


class Context:
    """One libdsort context bound to one GPU (dsort_init / dsort_finalize)."""

    def __init__(self, device=0):
        self.lib = load()
        h = P()
        rc = self.lib.dsort_init(ctypes.byref(h), device)
        if rc != DSORT_OK:
            raise DsortError(f"dsort_init(device={device}) failed: {rc} ({ERRORS.get(rc, '?')}); "
                             "a gfx950 GPU is required (no CPU fallback)")
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            self.lib.dsort_finalize(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc):
        return _check(self.h, rc)

    # ---------------- options (dsort_set_option) -----------------------------------------
    @staticmethod
    def _opt(name):
        return OPTIONS[name]  # (ABI 6 dropped ABI 2's "kill_after_pass" alias)

    def set_option(self, name, value):
        self.check(self.lib.dsort_set_option(self.h, self._opt(name), int(value)))

    def get_option(self, name):
        v = ctypes.c_int64()
        self.check(self.lib.dsort_get_option(self.h, self._opt(name), ctypes.byref(v)))
        return v.value

    @contextlib.contextmanager
    def options(self, **kw):
        """Sets options for the body of a with-statement and restores the previous values."""
        old = {k: self.get_option(k) for k in kw}
        try:
            for k, v in kw.items():
                self.set_option(k, v)
            yield self
        finally:
            for k, v in old.items():
                self.set_option(k, v)

    def sort_stages(self, n, key_bytes=4):
        """Kill points of a sort of n keys under this context's options (dsort_sort_stages)."""
        m = ctypes.c_int()
        self.check(self.lib.dsort_sort_stages(self.h, n, key_bytes, ctypes.byref(m)))
        return m.value

    # ---------------- host-buffer entry points (reference drop-ins) ----------------------
    def sort(self, keys):
        """In-place sort of a host numpy int32/int64 array (dsort_sort_*)."""
        assert keys.flags.c_contiguous
        f = getattr(self.lib, f"dsort_sort_{_sfx(keys.dtype)}")
        self.check(f(self.h, _ptr(keys), keys.size))
        return keys

    def merge(self, runs):
        """Merge sorted host runs (dsort_merge_*); returns a new array."""
        runs = [np.ascontiguousarray(r) for r in runs]
        dt = runs[0].dtype if runs else np.dtype(np.int32)
        k = len(runs)
        ptrs = (ctypes.c_void_p * max(k, 1))(*[r.ctypes.data for r in runs])
        lens = (ctypes.c_size_t * max(k, 1))(*[r.size for r in runs])
        out = np.empty(sum(r.size for r in runs), dt)
        f = getattr(self.lib, f"dsort_merge_{_sfx(dt)}")
        self.check(f(self.h, ctypes.cast(ptrs, P), ctypes.cast(lens, P), k, _ptr(out)))
        return out

    # ---------------- device entry points (torch tensors) --------------------------------
    @staticmethod
    def _stream():
        # torch's default stream is HIP's null stream (handle 0); NULL would select the
        # context's own non-blocking stream, which is not ordered with torch's work.
        h = torch.cuda.current_stream().cuda_stream
        return ctypes.c_void_p(h if h else 1)  # 1 == DSORT_NULL_STREAM

    @staticmethod
    def _tsfx(t):
        if t.dtype == torch.int32:
            return "i32"
        if t.dtype == torch.int64:
            return "i64"
        raise DsortError(f"unsupported tensor dtype {t.dtype}")

    def sort_dev(self, t, out=None):
        """Sort a CUDA tensor in place, or into `out` (dsort_sort_dev[_copy]_*)."""
        sfx = self._tsfx(t)
        if out is None:
            self.check(getattr(self.lib, f"dsort_sort_dev_{sfx}")(self.h, t.data_ptr(), t.numel(),
                                                                   self._stream()))
            return t
        assert out.numel() == t.numel() and out.dtype == t.dtype
        self.check(getattr(self.lib, f"dsort_sort_dev_copy_{sfx}")(self.h, t.data_ptr(), out.data_ptr(),
                                                                    t.numel(), self._stream()))
        return out

    def merge_dev(self, t, lens, out):
        sfx = self._tsfx(t)
        k = len(lens)
        la = (ctypes.c_size_t * max(k, 1))(*[int(x) for x in lens])
        self.check(getattr(self.lib, f"dsort_merge_dev_{sfx}")(self.h, t.data_ptr(), ctypes.cast(la, P), k,
                                                                out.data_ptr(), self._stream()))
        return out

    def gen_uniform(self, t, seed, first=0):
        sfx = self._tsfx(t)
        self.check(getattr(self.lib, f"dsort_gen_uniform_{sfx}")(self.h, t.data_ptr(), t.numel(), seed, first,
                                                                  self._stream()))
        return t

    def gen_zipf_i64(self, t, seed, first=0):
        assert t.dtype == torch.int64
        self.check(self.lib.dsort_gen_zipf_i64(self.h, t.data_ptr(), t.numel(), seed, first, self._stream()))
        return t

    def fingerprint(self, t, n=None):
        torch.cuda.current_stream().synchronize()
        s, x = U64(), U64()
        n = t.numel() if n is None else n
        self.check(getattr(self.lib, f"dsort_fingerprint_{self._tsfx(t)}")(self.h, t.data_ptr(), n,
                                                                            ctypes.byref(s), ctypes.byref(x)))
        return s.value, x.value

    def descents(self, t, n=None):
        torch.cuda.current_stream().synchronize()
        c = U64()
        n = t.numel() if n is None else n
        self.check(getattr(self.lib, f"dsort_count_descents_{self._tsfx(t)}")(self.h, t.data_ptr(), n,
                                                                               ctypes.byref(c)))
        return c.value

    def format_text(self, keys, text):
        """output.txt bytes of int32 CUDA tensor `keys` into uint8 CUDA tensor `text` (>= 12 bytes
        per key); returns the byte count (dsort_format_text_dev_i32)."""
        assert keys.dtype == torch.int32 and text.dtype == torch.uint8
        ln = ctypes.c_size_t()
        self.check(self.lib.dsort_format_text_dev_i32(self.h, keys.data_ptr(), keys.numel(), text.data_ptr(),
                                                      text.numel(), ctypes.byref(ln), self._stream()))
        return ln.value

    def parse_text(self, text, nbytes, keys):
        """Parse the first `nbytes` of uint8 CUDA tensor `text` (16-byte aligned) into int32 CUDA
        tensor `keys`; returns the token count (dsort_parse_text_dev_i32)."""
        assert keys.dtype == torch.int32 and text.dtype == torch.uint8 and nbytes <= text.numel()
        cnt = ctypes.c_size_t()
        self.check(self.lib.dsort_parse_text_dev_i32(self.h, text.data_ptr(), nbytes, keys.data_ptr(),
                                                     keys.numel(), ctypes.byref(cnt), self._stream()))
        return cnt.value

    def parse_text_host(self, raw):
        """Host bytes -> np.int32 keys through the GPU parser (dsort_parse_text_i32)."""
        cap = len(raw) // 2 + 1
        out = np.empty(cap, np.int32)
        cnt = ctypes.c_size_t()
        self.check(self.lib.dsort_parse_text_i32(self.h, raw, len(raw), _ptr(out), cap, ctypes.byref(cnt)))
        return out[:cnt.value]

    def format_text_host(self, keys):
        """np.int32 keys -> output.txt bytes through the GPU formatter (dsort_format_text_i32)."""
        keys = np.ascontiguousarray(keys, np.int32)
        buf = ctypes.create_string_buffer(12 * keys.size + 1)
        ln = ctypes.c_size_t()
        self.check(self.lib.dsort_format_text_i32(self.h, _ptr(keys), keys.size, buf, len(buf),
                                                  ctypes.byref(ln)))
        return buf.raw[:ln.value]

    def stats(self):
        st = Stats()
        self.check(self.lib.dsort_get_stats(self.h, ctypes.byref(st)))
        return st.as_dict()

    def synchronize(self):
        self.check(self.lib.dsort_synchronize(self.h))

    # ---------------- multi-GPU -----------------------------------------------------------
    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(128)
        _check(None, load().dsort_comm_unique_id(buf))
        return bytes(buf.raw)

    def comm_init(self, nranks, rank, uid):
        assert len(uid) == 128
        buf = ctypes.create_string_buffer(uid, 128)
        self.check(self.lib.dsort_comm_init(self.h, nranks, rank, buf))

    def comm_init_transport(self, nranks, rank, transport):
        self._transport = transport  # keep the callbacks alive while the library may call them
        if getattr(transport, "deadline_fn", None) is None:
            transport.deadline_fn = self.deadline_ms  # the callbacks' waits end at the exchange deadline
        self.check(self.lib.dsort_comm_init_transport(self.h, nranks, rank, ctypes.byref(transport)))

    def deadline_ms(self):
        """Milliseconds left before the running sample sort's exchange deadline, -1 for none
        (dsort_comm_deadline_ms; for transport callbacks on the sorting thread)."""
        v = ctypes.c_int64()
        self.check(self.lib.dsort_comm_deadline_ms(self.h, ctypes.byref(v)))
        return v.value

    def comm_destroy(self):
        self.check(self.lib.dsort_comm_destroy(self.h))

    def comm_abort(self):
        self.check(self.lib.dsort_comm_abort(self.h))

    def sample_sort_dev(self, t):
        """Returns (device pointer int, n_out) of this rank's slice (context-owned)."""
        sfx = self._tsfx(t)
        outp, nout = P(), SZ()
        self.check(getattr(self.lib, f"dsort_sample_sort_dev_{sfx}")(self.h, t.data_ptr(), t.numel(),
                                                                      ctypes.byref(outp), ctypes.byref(nout),
                                                                      self._stream()))
        return outp.value or 0, nout.value

    def sample_merge_dev(self, t):
        """Exchange half of the sample sort for an already sorted local run `t`
        (dsort_sample_merge_dev_*).  Returns (device pointer int, n_out) like sample_sort_dev."""
        sfx = self._tsfx(t)
        outp, nout = P(), SZ()
        self.check(getattr(self.lib, f"dsort_sample_merge_dev_{sfx}")(self.h, t.data_ptr(), t.numel(),
                                                                       ctypes.byref(outp), ctypes.byref(nout),
                                                                       self._stream()))
        return outp.value or 0, nout.value

    def copy_d2h(self, host, dptr, nbytes):
        self.check(self.lib.dsort_copy_d2h(self.h, _ptr(host), dptr, nbytes))
        return host

"""ctypes binding of ``libkmerpapa_hip.so`` (C-ABI in include/kmerpapa_hip.h).

This is the only door from the Python host layer into the GPU.  There is no CPU
fallback: if the HIP library is missing or no GPU is visible, :func:`load` / :class:`Device`
raise, loudly.

Host-side responsibilities kept here:
  * k-mer ordering: count tables go to the device in KmerEnumeration order (position 0
    fastest, nucleotide digit = index in ``code[g]``), see ``kmer_order``;
  * pass planning: lane groups are packed into passes that fit device memory
    (4 bytes per cell per lane: the f32 train score of the value-only sweep, plus a
    per-lane backtrack node pool; ``Plan.info["bytes_per_lane"]``);
  * sharding: groups are spread over the visible GPUs, one host thread per GPU
    (ctypes releases the GIL during every call), no collective needed.
"""
import atexit
import ctypes
import os
import threading
import time

import numpy as np

from .pattern_utils import code_no

_HERE = os.path.dirname(os.path.abspath(__file__))
# KMERPAPA_LIB selects another build of the same C-ABI (e.g. the -DKP_STAMPS diagnostic build)
LIB_PATH = os.environ.get("KMERPAPA_LIB") or os.path.join(_HERE, "libkmerpapa_hip.so")
MAX_GROUP_LANES = 8

_lib = None
_lib_lock = threading.Lock()


class KPError(RuntimeError):
    """Error reported by the C-ABI (carries the KP_E_* code)."""

    def __init__(self, code, msg):
        super().__init__(f"kmerpapa_hip error {code}: {msg}")
        self.code = code


class KPGroup(ctypes.Structure):
    _fields_ = [("fold", ctypes.c_int32), ("n_lanes", ctypes.c_int32), ("alpha", ctypes.c_double),
                ("beta", ctypes.c_double), ("penalty", ctypes.c_double * MAX_GROUP_LANES)]


class KPPlanInfo(ctypes.Structure):
    _fields_ = [("npat", ctypes.c_uint64), ("nblocks", ctypes.c_uint64), ("n_kmers", ctypes.c_uint64),
                ("block", ctypes.c_uint32), ("block_pad", ctypes.c_uint32), ("k", ctypes.c_int32),
                ("low_positions", ctypes.c_int32), ("max_level", ctypes.c_int32),
                ("high_levels", ctypes.c_int32), ("pairs_total", ctypes.c_double),
                ("pairs_high", ctypes.c_double), ("bytes_per_lane", ctypes.c_uint64),
                ("lanes_per_workgroup", ctypes.c_uint32), ("pad_", ctypes.c_uint32)]


class KPPassStats(ctypes.Structure):
    _fields_ = [("dp_ms", ctypes.c_double), ("backtrack_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("units", ctypes.c_uint64), ("dp_launches", ctypes.c_uint64), ("alg_bytes", ctypes.c_double),
                ("gather_bytes", ctypes.c_double)]


EXPORTS = ["kp_last_error", "kp_device_count", "kp_create", "kp_destroy", "kp_device_mem", "kp_plan_create",
           "kp_plan_destroy", "kp_plan_get_info", "kp_plan_host", "kp_plan_host_counts", "kp_set_counts", "kp_counts_begin", "kp_counts_fold", "kp_pass",
           "kp_reserve_lanes", "kp_last_pass_stats", "kp_last_launch_ms", "kp_fit_leaves", "kp_dump_lane", "kp_gather_cells", "kp_fold_split",
           "kp_fold_sample", "kp_math_log", "kp_math_libm", "kp_kmer_parse", "kp_kmer_table_info", "kp_kmer_table_copy", "kp_kmer_table_free",
           "kp_format_long_rows", "kp_py_repr", "kp_device_groups", "kp_allkmers_cv", "kp_block_order_check",
           "kp_plan_block_check"]


def load():
    """Load libkmerpapa_hip.so (built in-tree by __graft_entry__.build())."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                              "g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.kp_last_error.restype = ctypes.c_char_p
        L.kp_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.kp_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
        L.kp_destroy.argtypes = [vp]
        L.kp_destroy.restype = None
        L.kp_device_mem.argtypes = [vp, u64p, u64p]
        L.kp_plan_create.argtypes = [vp, ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(vp)]
        L.kp_plan_destroy.argtypes = [vp]
        L.kp_plan_destroy.restype = None
        L.kp_plan_get_info.argtypes = [vp, ctypes.POINTER(KPPlanInfo)]
        L.kp_plan_host.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(KPPlanInfo)]
        if hasattr(L, "kp_plan_host_counts"):  # (older builds loaded through KMERPAPA_LIB for A/B timing lack it)
            L.kp_plan_host_counts.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int,
                                              ctypes.POINTER(KPPlanInfo)]
        L.kp_block_order_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32, u64p]
        L.kp_plan_block_check.argtypes = [vp, u64p]
        L.kp_kmer_parse.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                    ctypes.POINTER(vp)]
        L.kp_kmer_table_info.argtypes = [vp, u64p, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64),
                                         ctypes.POINTER(ctypes.c_int64)]
        L.kp_kmer_table_copy.argtypes = [vp, vp, vp, vp]
        L.kp_kmer_table_free.argtypes = [vp]
        L.kp_kmer_table_free.restype = None
        L.kp_set_counts.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
        L.kp_counts_begin.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
        L.kp_counts_fold.argtypes = [vp, ctypes.c_int, vp, vp, ctypes.c_uint64]
        L.kp_pass.argtypes = [vp, ctypes.POINTER(KPGroup), ctypes.c_int, vp, vp, vp]
        L.kp_last_pass_stats.argtypes = [vp, ctypes.POINTER(KPPassStats)]
        L.kp_device_groups.argtypes = [ctypes.POINTER(KPGroup), ctypes.c_int, ctypes.c_int, vp, vp, vp, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int)]
        L.kp_last_launch_ms.argtypes = [vp, vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.kp_reserve_lanes.argtypes = [vp, ctypes.c_uint32]
        L.kp_fit_leaves.argtypes = [vp, ctypes.c_uint32, vp, ctypes.c_uint64, u64p]
        L.kp_dump_lane.argtypes = [vp, ctypes.c_uint32, vp, vp]
        L.kp_gather_cells.argtypes = [vp, ctypes.c_uint32, vp, ctypes.c_uint64, vp]
        L.kp_fold_split.argtypes = [vp, ctypes.POINTER(ctypes.c_int32), vp, ctypes.c_uint64, ctypes.c_int, vp]
        if hasattr(L, "kp_math_log"):  # (older builds loaded through KMERPAPA_LIB for A/B timing lack it)
            L.kp_math_log.argtypes = [vp, vp, vp, ctypes.c_uint64]
        if hasattr(L, "kp_math_libm"):
            L.kp_math_libm.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.c_int]
        L.kp_format_long_rows.argtypes = [vp, ctypes.c_int, vp, vp, vp, ctypes.c_uint64, vp, vp, ctypes.c_uint64, vp,
                                          ctypes.c_uint64, u64p]
        L.kp_py_repr.argtypes = [vp, ctypes.c_uint64, vp, ctypes.c_uint64, u64p]
        L.kp_allkmers_cv.argtypes = [vp, vp, vp, ctypes.c_uint64, ctypes.c_int, vp, vp, ctypes.c_int, vp, vp]
        L.kp_fold_sample.argtypes = [vp, ctypes.POINTER(ctypes.c_int32), vp, ctypes.c_uint64, ctypes.c_uint64, vp]
        for name in EXPORTS:
            if not hasattr(L, name):
                continue
            if name not in ("kp_destroy", "kp_plan_destroy", "kp_last_error", "kp_kmer_table_free"):
                getattr(L, name).restype = ctypes.c_int
        _lib = L
        return L


def _check(rc):
    if rc != 0:
        raise KPError(rc, load().kp_last_error().decode(errors="replace"))


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


# launch knobs read by kp_hip.hip (every setting gives the same scores; they change timing)
LAUNCH_KNOBS = ("KP_DP_THREADS", "KP_LANES_PER_WG", "KP_XCD_REMAP", "KP_LANE_SPLIT", "KP_NT_STORE", "KP_NT_SLOW",
                "KP_BLOCK_PERM", "KP_BLOCK_ORDER", "KP_BLOCK_TILE", "KP_LOW_ORDER", "KP_EXACT_LOGS",
               "KP_CLASS_STREAMS", "KP_NT_SLOW_H", "KP_LDS_BUDGET", "KP_WIDE_SPLIT", "KP_HPD", "KP_WS")


_toolchain = None


def toolchain_version():
    """``hipcc --version`` of the compiler that built the library, recorded by the build
    (csrc/kp_toolchain.txt; part of kernel_tag)."""
    global _toolchain
    if _toolchain is None:
        try:
            with open(os.path.join(_HERE, "csrc", "kp_toolchain.txt")) as f:
                _toolchain = f.read()
        except OSError:
            _toolchain = "toolchain: not recorded (library not built by csrc/Makefile)"
    return _toolchain


def kernel_tag():
    """Short hash of everything that decides the sweep's launches: the library's tracked
    sources (csrc/kp_*.h, kp_*.hip, gen_logdata.py, Makefile, the C-ABI header), the log
    constants generated into kp_logdata.h (without its comment lines, which name the host
    libm's path), the compiler (``hipcc --version``) and the launch knobs set in the
    environment.  Ties PMC profiles (profiles/*/pmc_*.json) to the exact build and launch
    configuration."""
    import glob
    import hashlib
    h = hashlib.sha1()
    csrc = os.path.join(_HERE, "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "kp_*.h")) + glob.glob(os.path.join(csrc, "kp_*.hip")))
    files = [f for f in files if os.path.basename(f) != "kp_logdata.h"]
    files += [os.path.join(csrc, "gen_logdata.py"), os.path.join(csrc, "Makefile"),
              os.path.join(os.path.dirname(_HERE), "include", "kmerpapa_hip.h")]
    for fn in files:
        if not os.path.isfile(fn):  # (an installed copy may lack a build file: hash its absence)
            h.update(b"missing:" + os.path.basename(fn).encode())
            continue
        with open(fn, "rb") as f:
            h.update(os.path.basename(fn).encode() + b"\0" + f.read())
    gen = os.path.join(csrc, "kp_logdata.h")
    if os.path.isfile(gen):
        with open(gen, "rb") as f:
            h.update(b"kp_logdata.h\0" + b"".join(x for x in f.readlines() if not x.lstrip().startswith(b"//")))
    h.update(toolchain_version().encode())
    for k in LAUNCH_KNOBS:
        h.update(f"{k}={os.environ.get(k, '')}".encode())
    return h.hexdigest()[:12]


def fold_split(colors, n_folds, prng):
    """Fold split of ``colors`` with the caller's numpy ``RandomState`` stream, in C++
    (``kp_fold_split``; bit-identical to CV_tools.py:5-62).  ``prng`` is advanced exactly
    as numpy's own draws would advance it.  Returns uint64 ``[n, n_folds]``."""
    L = load()
    st = prng.get_state(legacy=True)
    if st[0] != "MT19937":
        raise ValueError("fold split needs a legacy MT19937 RandomState")
    key = np.array(st[1], dtype=np.uint32)
    pos = ctypes.c_int32(int(st[2]))
    col = np.ascontiguousarray(colors, dtype=np.uint64)
    out = np.zeros((col.shape[0], int(n_folds)), dtype=np.uint64)
    _check(L.kp_fold_split(_ptr(key), ctypes.byref(pos), _ptr(col), ctypes.c_uint64(col.shape[0]), int(n_folds),
                           _ptr(out)))
    prng.set_state((st[0], key, pos.value, st[3], st[4]))
    return out


def fold_sample(colors, m, prng):
    """One fold of the split: ``m`` balls drawn colour by colour from ``colors``
    (CV_tools.py sample :5-27) with the caller's numpy ``RandomState`` stream, in C++
    (``kp_fold_sample``).  Returns uint64 ``[n]``; ``prng`` advances as numpy's would."""
    L = load()
    st = prng.get_state(legacy=True)
    if st[0] != "MT19937":
        raise ValueError("fold split needs a legacy MT19937 RandomState")
    key = np.array(st[1], dtype=np.uint32)
    pos = ctypes.c_int32(int(st[2]))
    col = np.ascontiguousarray(colors, dtype=np.uint64)
    out = np.zeros(col.shape[0], dtype=np.uint64)
    _check(L.kp_fold_sample(_ptr(key), ctypes.byref(pos), _ptr(col), ctypes.c_uint64(col.shape[0]),
                            ctypes.c_uint64(int(m)), _ptr(out)))
    prng.set_state((st[0], key, pos.value, st[3], st[4]))
    return out


def parse_kmer_counts(text, columns, super_pattern=None, length=0):
    """Parse k-mer count text with the native reader (``kp_kmer_parse``, C++).

    ``text``: bytes of a "kmer count" (``columns=2``) or "kmer positive background"
    (``columns=3``) file.  Returns ``(k, codes uint64, c0 int64, c1 int64, total0,
    total1)`` with codes sorted (2 bits per letter, first letter most significant).
    Input errors raise ``ValueError`` with the parser's message."""
    L = load()
    buf = bytes(text)
    t = ctypes.c_void_p()
    sp = super_pattern.encode("ascii") if super_pattern else None
    rc = L.kp_kmer_parse(buf, ctypes.c_uint64(len(buf)), int(columns), sp, int(length or 0), ctypes.byref(t))
    if rc != 0:
        raise ValueError(L.kp_last_error().decode(errors="replace"))
    try:
        n, k = ctypes.c_uint64(), ctypes.c_int32()
        t0, t1 = ctypes.c_int64(), ctypes.c_int64()
        _check(L.kp_kmer_table_info(t, ctypes.byref(n), ctypes.byref(k), ctypes.byref(t0), ctypes.byref(t1)))
        codes = np.zeros(n.value, np.uint64)
        c0 = np.zeros(n.value, np.int64)
        c1 = np.zeros(n.value, np.int64)
        _check(L.kp_kmer_table_copy(t, _ptr(codes), _ptr(c0), _ptr(c1)))
    finally:
        L.kp_kmer_table_free(t)
    return k.value, codes, c0, c1, t0.value, t1.value


def py_repr(x):
    """Python repr() of every float64 in ``x`` by the native formatter (kp_py_repr); a list
    of str.  Host code, no GPU (a check of kp_format_long_rows' float format)."""
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
    cap = 40 * x.size + 1
    buf = ctypes.create_string_buffer(cap)
    n = ctypes.c_uint64()
    _check(load().kp_py_repr(_ptr(x), ctypes.c_uint64(x.size), buf, ctypes.c_uint64(cap), ctypes.byref(n)))
    return buf.raw[:n.value].decode("ascii").split("\n")[:-1]


def format_long_rows(kmers, c_neg, c_pos, pid, tails):
    """The -l output rows (kp_format_long_rows): ``kmers`` uint8 ``[n, k]`` letters,
    ``c_neg``/``c_pos`` int64 ``[n]``, ``pid`` ``[n]`` = index into ``tails`` (list of
    str, each " pattern p_neg p_pos p_rate\n").  Returns the text as bytes; a row with no
    counts raises ZeroDivisionError, as the reference's formula does."""
    kmers = np.ascontiguousarray(kmers, dtype=np.uint8)
    n, k = kmers.shape
    c_neg = np.ascontiguousarray(c_neg, dtype=np.int64)
    c_pos = np.ascontiguousarray(c_pos, dtype=np.int64)
    pid = np.ascontiguousarray(pid, dtype=np.uint32)
    tb = [t.encode("ascii") for t in tails]
    off = np.zeros(len(tb) + 1, np.uint64)
    off[1:] = np.cumsum([len(t) for t in tb])
    tail_bytes = b"".join(tb) or b"\0"
    lens = np.array([len(t) for t in tb] or [0], np.int64)
    cap = int(n * (k + 3 * 32) + (lens[pid].sum() if n else 0)) + 1
    out = np.empty(cap, np.uint8)  # (not zeroed: only the w bytes written are returned)
    w = ctypes.c_uint64()
    rc = load().kp_format_long_rows(kmers.ctypes.data_as(ctypes.c_void_p), int(k), _ptr(c_neg), _ptr(c_pos),
                                    _ptr(pid), ctypes.c_uint64(n), tail_bytes, _ptr(off), ctypes.c_uint64(len(tb)),
                                    _ptr(out), ctypes.c_uint64(cap), ctypes.byref(w))
    if rc != 0:
        msg = load().kp_last_error().decode(errors="replace")
        if "division by zero" in msg:
            raise ZeroDivisionError("float division by zero")
        raise KPError(rc, msg)
    return out[:w.value].tobytes()


def plan_info(gen_pat, max_block=0):
    """The plan's info (cells, blocks, device bytes per lane, ...) built on the host only
    (kp_plan_host): no GPU is touched."""
    info = KPPlanInfo()
    _check(load().kp_plan_host(gen_pat.encode(), ctypes.c_uint32(max_block), ctypes.byref(info)))
    return {name: getattr(info, name) for name, _ in KPPlanInfo._fields_}


def shard_width(gen_pat, itype=np.uint32, max_block=0):
    """Lanes one sweep workgroup holds for ``gen_pat``'s lattice at count width ``itype``
    (kp_plan_host_counts, host only): the group size shard.assign_lanes deals whole.  A pure
    function of the lattice and the count width, so every rank of a job computes the same."""
    info = KPPlanInfo()
    _check(load().kp_plan_host_counts(gen_pat.encode(), ctypes.c_uint32(max_block), int(np.dtype(itype).itemsize),
                                      ctypes.byref(info)))
    return int(info.lanes_per_workgroup)


def counts_itype(M):
    """Count width of a run's counts: an array, a FoldFeed, or None (uint32)."""
    if isinstance(M, FoldFeed):
        return M.M_all.dtype
    return np.asarray(M).dtype if M is not None else np.dtype(np.uint32)


def block_order_check(gen_pat, max_block=0):
    """Blocks of ``gen_pat``'s lattice whose closed-form block-list slot (the rule the
    device builds the list by, kp_blocks_kernel) differs from the host's block walk
    (kp_block_order_check, host code): 0 when the two agree."""
    n = ctypes.c_uint64()
    _check(load().kp_block_order_check(gen_pat.encode(), ctypes.c_uint32(max_block), ctypes.byref(n)))
    return n.value


def _group_array(groups):
    """``groups`` (list of ``(fold, alpha, beta, penalties)``; ``beta`` may be a callable) as
    the C-ABI's kp_group array; returns it and the number of lanes."""
    arr = (KPGroup * len(groups))()
    nl = 0
    for i, (fold, alpha, beta, pens) in enumerate(groups):
        pens = list(pens)
        if not 1 <= len(pens) <= MAX_GROUP_LANES:
            raise ValueError("a group holds 1..8 penalties")
        arr[i].fold = int(fold)
        arr[i].n_lanes = len(pens)
        arr[i].alpha = float(alpha)
        arr[i].beta = float(beta() if callable(beta) else beta)
        for j, c in enumerate(pens):
            arr[i].penalty[j] = float(c)
        nl += len(pens)
    return arr, nl


def device_groups(groups, width):
    """The workgroups (device groups) kp_pass runs ``groups`` as, at ``width`` lanes per
    workgroup (kp_device_groups, host code): a list of ``(lane0, lanes, mixed_lanes)``."""
    arr, nl = _group_array(groups)
    cap = nl
    lane0 = np.zeros(cap, np.int32)
    nls = np.zeros(cap, np.int32)
    nl2 = np.zeros(cap, np.int32)
    n = ctypes.c_int()
    _check(load().kp_device_groups(arr, len(groups), width, _ptr(lane0), _ptr(nls), _ptr(nl2), cap, ctypes.byref(n)))
    return [(int(lane0[i]), int(nls[i]), int(nl2[i])) for i in range(n.value)]


def device_count():
    n = ctypes.c_int(0)
    _check(load().kp_device_count(ctypes.byref(n)))
    return n.value


def visible_devices():
    """GPUs the DP may use: $KMERPAPA_DEVICES (comma list) or every visible device."""
    env = os.environ.get("KMERPAPA_DEVICES")
    if env:
        return [int(x) for x in env.split(",") if x.strip()]
    return list(range(device_count()))


class Device:
    """One HIP device context (stream + events) of the library."""

    def __init__(self, device=0):
        L = load()
        self.device = device
        self._h = ctypes.c_void_p()
        _check(L.kp_create(int(device), ctypes.byref(self._h)))

    def mem(self):
        fr, tot = ctypes.c_uint64(), ctypes.c_uint64()
        _check(load().kp_device_mem(self._h, ctypes.byref(fr), ctypes.byref(tot)))
        return fr.value, tot.value

    def log(self, x):
        """float64 log of every element on this GPU (kp_math_log: the DP's device log)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.empty_like(x)
        _check(load().kp_math_log(self._h, _ptr(x), _ptr(y), ctypes.c_uint64(x.size)))
        return y

    def libm(self, x, fn):
        """The C library's log (fn 1) or log1p (fn 2) as the GPU computes it (kp_math_libm)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.empty_like(x)
        _check(load().kp_math_libm(self._h, _ptr(x), _ptr(y), ctypes.c_uint64(x.size), int(fn)))
        return y

    def allkmers_cv(self, M, U, alphas, betas):
        """--score all_kmers on this GPU (kp_allkmers_cv; all_kmers_CV.py :8-46): ``M``/``U``
        ``[n, nf]`` fold counts (rows in matches(gen_pat) order), ``betas`` ``[na, nf]``.
        Returns ``(sum_train, sum_test)`` ``[na, nf]`` float64, each summed k-mer by k-mer
        as the reference does."""
        M = np.ascontiguousarray(M, dtype=np.uint64)
        U = np.ascontiguousarray(U, dtype=np.uint64)
        if M.ndim != 2 or U.shape != M.shape:
            raise ValueError("counts must be [n_kmers, nfolds]")
        al = np.ascontiguousarray(alphas, dtype=np.float64).reshape(-1)
        be = np.ascontiguousarray(betas, dtype=np.float64).reshape(al.size, M.shape[1])
        tr = np.zeros(be.shape, np.float64)
        te = np.zeros(be.shape, np.float64)
        _check(load().kp_allkmers_cv(self._h, _ptr(M), _ptr(U), ctypes.c_uint64(M.shape[0]), int(M.shape[1]),
                                     _ptr(al), _ptr(be), int(al.size), _ptr(tr), _ptr(te)))
        return tr, te

    def close(self):
        if self._h:
            load().kp_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Plan:
    """The lattice of one general pattern on one device, with its resident buffers."""

    def __init__(self, device, gen_pat, max_block=0):
        self.device = device
        self.gen_pat = gen_pat
        self._h = ctypes.c_void_p()
        _check(load().kp_plan_create(device._h, gen_pat.encode(), ctypes.c_uint32(max_block), ctypes.byref(self._h)))
        info = KPPlanInfo()
        _check(load().kp_plan_get_info(self._h, ctypes.byref(info)))
        self.info = {name: getattr(info, name) for name, _ in KPPlanInfo._fields_}
        self.nf = None
        self.itype = None
        self.last_lanes = 0
        self.lanes_held = 0  # lanes the device buffers hold (they only grow)

    def set_counts(self, M, U):
        """Fold counts ``[n_kmers, nf]`` (uint32/uint64) in KmerEnumeration order."""
        M = np.ascontiguousarray(M)
        if M.dtype not in (np.uint32, np.uint64):
            raise TypeError("counts must be uint32 or uint64")
        U = np.ascontiguousarray(U, dtype=M.dtype)
        if M.ndim == 1:
            M = M.reshape(-1, 1)
            U = U.reshape(-1, 1)
        _check(load().kp_set_counts(self._h, _ptr(M), _ptr(U), ctypes.c_uint64(M.shape[0]), int(M.shape[1]),
                                    int(M.dtype.itemsize)))
        self.nf = M.shape[1]
        self.itype = M.dtype
        self._refresh_info()

    def _refresh_info(self):
        """Re-read the plan's info: lanes_per_workgroup depends on the count width, fixed
        once counts are set (64-bit counts above 2^32 - 1 take more LDS)."""
        info = KPPlanInfo()
        _check(load().kp_plan_get_info(self._h, ctypes.byref(info)))
        self.info = {name: getattr(info, name) for name, _ in KPPlanInfo._fields_}

    def counts_begin(self, M_all, U_all, nf):
        """Start a fold-by-fold count upload: ``M_all``/``U_all`` ``[n_kmers]`` = counts of
        all data in k-mer order (uint32/uint64), ``nf`` folds to come (kp_counts_begin)."""
        M_all = np.ascontiguousarray(M_all).reshape(-1)
        if M_all.dtype not in (np.uint32, np.uint64):
            raise TypeError("counts must be uint32 or uint64")
        U_all = np.ascontiguousarray(U_all, dtype=M_all.dtype).reshape(-1)
        _check(load().kp_counts_begin(self._h, _ptr(M_all), _ptr(U_all), ctypes.c_uint64(M_all.shape[0]), int(nf),
                                      int(M_all.dtype.itemsize)))
        self.nf = int(nf)
        self.itype = M_all.dtype
        self._refresh_info()

    def counts_fold(self, fold, M_fold, U_fold):
        """Counts of one fold ``[n_kmers]`` (same itype as counts_begin; kp_counts_fold)."""
        M_fold = np.ascontiguousarray(M_fold, dtype=self.itype).reshape(-1)
        U_fold = np.ascontiguousarray(U_fold, dtype=self.itype).reshape(-1)
        _check(load().kp_counts_fold(self._h, int(fold), _ptr(M_fold), _ptr(U_fold), ctypes.c_uint64(M_fold.shape[0])))

    def run(self, groups):
        """One DP sweep.  ``groups``: list of ``(fold, alpha, beta, penalties)``; ``beta`` may
        be a callable returning it (the CV driver's betas of folds still being drawn).

        Returns ``(root_train f32[L], root_test f32[L], n_leaves u64[L])`` with lanes
        numbered group-major.
        """
        arr, nl = _group_array(groups)
        rt = np.zeros(nl, np.float32)
        re = np.zeros(nl, np.float32)
        nlv = np.zeros(nl, np.uint64)
        _check(load().kp_pass(self._h, arr, len(groups), _ptr(rt), _ptr(re), _ptr(nlv)))
        self.last_lanes = nl
        self.lanes_held = max(self.lanes_held, nl)
        return rt, re, nlv

    def reserve(self, lanes):
        """Allocate the per-lane buffers for ``lanes`` lanes now (kp_reserve_lanes)."""
        _check(load().kp_reserve_lanes(self._h, int(lanes)))
        self.lanes_held = max(self.lanes_held, int(lanes))

    def stats(self):
        s = KPPassStats()
        _check(load().kp_last_pass_stats(self._h, ctypes.byref(s)))
        return {name: getattr(s, name) for name, _ in KPPassStats._fields_}

    def block_check(self):
        """Entries of the device block list (built by kp_blocks_kernel) that differ from the
        host's block walk (kp_plan_block_check): 0 when they agree."""
        n = ctypes.c_uint64()
        _check(load().kp_plan_block_check(self._h, ctypes.byref(n)))
        return n.value

    def launch_ms(self):
        """Per-launch device times (ms) of the last pass (needs KP_LAUNCH_TIMES=1)."""
        n = ctypes.c_int()
        _check(load().kp_last_launch_ms(self._h, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, np.float32)
        _check(load().kp_last_launch_ms(self._h, _ptr(out), n.value, ctypes.byref(n)))
        return out

    def leaves(self, lane):
        """Cell indices of the optimal partition of ``lane``, in backtrack order."""
        n = ctypes.c_uint64()
        _check(load().kp_fit_leaves(self._h, int(lane), None, ctypes.c_uint64(0), ctypes.byref(n)))
        out = np.zeros(max(1, n.value), np.uint64)
        _check(load().kp_fit_leaves(self._h, int(lane), _ptr(out), ctypes.c_uint64(out.size), ctypes.byref(n)))
        return out[:n.value]

    def dump_lane(self, lane):
        score = np.zeros(self.info["npat"], np.float32)
        code = np.zeros(self.info["npat"], np.uint8)
        _check(load().kp_dump_lane(self._h, int(lane), _ptr(score), _ptr(code)))
        return score, code

    def gather_cells(self, lane, cells):
        """Train scores (f32) of the cells ``cells`` (uint64 indices) of ``lane`` of the last
        pass (kp_gather_cells)."""
        cells = np.ascontiguousarray(cells, dtype=np.uint64).reshape(-1)
        out = np.zeros(cells.size, np.float32)
        _check(load().kp_gather_cells(self._h, int(lane), _ptr(cells), ctypes.c_uint64(cells.size), _ptr(out)))
        return out

    def lanes_that_fit(self, reserve=2 << 30):
        fr, _ = self.device.mem()
        per = self.info["bytes_per_lane"]
        # the lane buffers already held are reused: count them as available
        held = self.lanes_held * per
        return max(0, int((fr + held - reserve) // per))

    def require_lanes(self, n=1, reserve=2 << 30):
        """Lanes that fit device memory now (``lanes_that_fit``); raises :class:`KPError`
        (KP_E_NOMEM) naming the lattice, its bytes per lane and the GPU's free memory if
        not even ``n`` do -- the reference would allocate its ``[npat, nf]`` arrays anyway
        (CV :93-102) and fail in numpy; a pass of zero lanes is never planned."""
        fit = self.lanes_that_fit(reserve)
        if fit < n:
            fr, tot = self.device.mem()
            per = self.info["bytes_per_lane"]
            raise KPError(-2, f"the lattice of {self.gen_pat} ({self.info['npat']:,} cells) needs "
                              f"{per / 1e9:.4g} GB of device memory per lane (float32 score per cell), "
                              f"{n} lane(s) at least; GPU {self.device.device} has {(fr + self.lanes_held * per) / 1e9:.4g} "
                              f"of {tot / 1e9:.4g} GB free after the plan's tables, of which {reserve / 2**30:.3g} GiB "
                              f"stay free for the library's working buffers. Restrict the general pattern "
                              f"with --super_pattern.")
        return fit

    def close(self):
        if self._h:
            load().kp_plan_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ----------------------------------------------------------------------------
# host helpers
# ----------------------------------------------------------------------------

def kmer_order(gen_pat, contexts):
    """KmerEnumeration index of every k-mer in ``contexts`` (vectorised): a list of k-mer
    strings, or a table with ``letters()`` (io_utils.KmerCounts, native parser output)."""
    k = len(gen_pat)
    if hasattr(contexts, "letters"):
        raw, name = contexts.letters(), contexts.kmer_at
    elif not contexts:
        return np.zeros(0, np.int64)
    else:
        raw = np.frombuffer("".join(contexts).encode("ascii"), dtype=np.uint8).reshape(len(contexts), k)
        name = contexts.__getitem__
    if raw.shape[0] == 0:
        return np.zeros(0, np.int64)
    idx = np.zeros(len(contexts), np.int64)
    w = 1
    for i, g in enumerate(gen_pat):
        lut = np.full(256, -1, np.int64)
        for nuc, d in code_no[g].items():
            lut[ord(nuc)] = d
        dig = lut[raw[:, i]]
        if (dig < 0).any():
            bad = name(int(np.argmax(dig < 0)))
            raise ValueError(f"k-mer {bad} does not match general pattern {gen_pat}")
        idx += dig * w
        w *= len(code_no[g])
    return idx


def counts_in_kmer_order(gen_pat, contexts, M, U, n_kmers, itype):
    """Scatter per-context rows ``[n, nf]`` into dense KmerEnumeration order (missing k-mers = 0)."""
    M = np.asarray(M)
    nf = 1 if M.ndim == 1 else M.shape[1]
    outM = np.zeros((n_kmers, nf), dtype=itype)
    outU = np.zeros((n_kmers, nf), dtype=itype)
    idx = kmer_order(gen_pat, contexts if hasattr(contexts, "letters") else list(contexts))
    outM[idx] = np.asarray(M, dtype=itype).reshape(len(idx), nf)
    outU[idx] = np.asarray(U, dtype=itype).reshape(len(idx), nf)
    return outM, outU


class FoldFeed:
    """Fold counts that arrive one fold at a time, in k-mer order: the CV driver draws the
    fold split on a host thread (CV_tools.fold_stream) while the GPUs already run the
    passes of the folds drawn so far.  ``M_all``/``U_all`` ``[n_kmers]`` = counts of all
    data (the sum of the folds to come), ``nf`` folds."""

    def __init__(self, M_all, U_all, nf):
        self.M_all = np.ascontiguousarray(M_all).reshape(-1)
        self.U_all = np.ascontiguousarray(U_all, dtype=self.M_all.dtype).reshape(-1)
        self.nf = int(nf)
        self._cols = [None] * self.nf
        self.t_put = [None] * self.nf  # perf_counter() at each fold's arrival
        self._err = None
        self._cv = threading.Condition()

    def put(self, fold, M_fold, U_fold):
        with self._cv:
            self._cols[fold] = (np.ascontiguousarray(M_fold, dtype=self.M_all.dtype),
                                np.ascontiguousarray(U_fold, dtype=self.M_all.dtype))
            self.t_put[fold] = time.perf_counter()
            self._cv.notify_all()

    def fail(self, exc):
        """The producer failed: every waiting and later ``get`` raises."""
        with self._cv:
            self._err = exc
            self._cv.notify_all()

    def get(self, fold):
        """``(M_fold, U_fold)``, waiting until the fold has been drawn."""
        with self._cv:
            while self._cols[fold] is None and self._err is None:
                self._cv.wait()
            if self._cols[fold] is None:
                raise RuntimeError(f"fold split failed before fold {fold}") from self._err
            return self._cols[fold]

    def arrays(self):
        """``(M, U)`` ``[n_kmers, nf]`` once every fold has arrived."""
        cols = [self.get(f) for f in range(self.nf)]
        return np.stack([c[0] for c in cols], axis=1), np.stack([c[1] for c in cols], axis=1)


def materialize(M, U, groups):
    """For runners without fold-by-fold upload: wait for a FoldFeed's folds and resolve
    callable betas.  Returns ``(M, U, groups)`` with arrays and float betas."""
    if isinstance(M, FoldFeed):
        M, U = M.arrays()
    groups = [(f, a, float(b() if callable(b) else b), pens) for f, a, b, pens in groups]
    return M, U, groups


# lanes a pass may hold when it packs groups of different widths (KMERPAPA_PASS_LANES; 0 =
# one sweep workgroup's width + 1, Plan.info["lanes_per_workgroup"] + 1)
PASS_LANES = int(os.environ.get("KMERPAPA_PASS_LANES", "0"))


def pass_cap(groups, fit, width=0):
    """Lanes per pass: PASS_LANES, by default one workgroup's ``width`` + 1 (6 at 9-mers),
    or the largest group if wider, if that fits.  A pass of two device groups runs their
    workgroups side by side in the same launches, so packing a small piece beside a full
    one saves the small pass's fixed work: 9-mer 5 + 1 lanes 468 ms against 371 + 108, 4 + 2
    482 against 310 + 182, 3 + 3 473 against 2 x 242 (profiles/r05/experiments/
    pack_lanes.txt) -- the pieces a lane-granular multi-GPU share is left with.  Wider packs
    gain less (5 + 2: 549 against 553) and every lane of the widest pass is allocated for the
    whole job (30.8 GB per lane at 9-mers), so one extra lane is the default.  The
    allocation's cost is the driver's wipe of HBM that earlier processes freed:
    about as long for 154 as for 185 GB when HBM is still being wiped, ~1 ms for either when
    it is clean.  Two 5-lane groups never share a pass: they are not faster per lane."""
    widest = max([len(g[3]) for g in groups] or [1])
    cap = PASS_LANES or ((width + 1) if width else 7)
    return min(fit, max(cap, widest))


def pack_passes(groups, max_lanes):
    """Split a group list into passes of at most ``max_lanes`` lanes (order kept)."""
    if max_lanes < 1:
        raise KPError(-2, "the lattice does not fit device memory even for one lane")
    passes, cur, n = [], [], 0
    for grp in groups:
        lanes = len(grp[3])
        if cur and n + lanes > max_lanes:
            passes.append(cur)
            cur, n = [], 0
        cur.append(grp)
        n += lanes
    if cur:
        passes.append(cur)
    return passes


def fold_pieces(groups, width):
    """The lanes of ``groups`` cut into pieces of at most ``width`` lanes, fold by fold: each
    fold's lanes (its groups in order, group-major) are cut together, so one piece may hold
    the last penalties of one alpha and the first of the next.  The library runs such a
    piece as ONE device group (a mixed group: the fold's count tables are shared, only the
    logs differ per alpha), so a 7-penalty grid runs as 5-lane workgroups instead of 5 + 2
    per alpha.  Returns pieces in order of first appearance of their fold; a piece is a list
    of ``(fold, alpha, beta, penalties, lane_ids)``, lane ids = group-major lane numbers in
    ``groups``."""
    start = np.cumsum([0] + [len(g[3]) for g in groups])
    folds = {}
    for gi, g in enumerate(groups):
        folds.setdefault(g[0], []).extend((gi, j) for j in range(len(g[3])))
    pieces = []
    for lanes in folds.values():
        for q in range(0, len(lanes), width):
            piece = []
            for gi, j in lanes[q:q + width]:
                f, a, b, pens = groups[gi][:4]
                if piece and piece[-1][5] == gi:
                    piece[-1][3].append(pens[j])
                    piece[-1][4].append(int(start[gi] + j))
                else:
                    piece.append([f, a, b, [pens[j]], [int(start[gi] + j)], gi])
            pieces.append([tuple(x[:5]) for x in piece])
    return pieces


def plan_passes(groups, max_lanes, width=None):
    """The passes one GPU runs for ``groups``, in run order: lowest fold first (folds are
    drawn in order, CV_tools.fold_stream, so the first pass starts as soon as the share's
    lowest fold is drawn), at most ``max_lanes`` lanes per pass.  With ``width`` (the lanes
    of one sweep workgroup, ``Plan.info["lanes_per_workgroup"]``) the lanes are first cut
    into fold pieces of that width (fold_pieces); without it every group is one piece.
    Pieces are packed in descending fold order and the passes then reversed, so a small
    piece (e.g. a 1-lane piece of a split group) joins the pass of a piece with the same or
    a HIGHER fold and never delays an earlier one.  Returns ``(passes, lane_order)``: a
    pass is a list of groups ``(fold, alpha, beta, penalties)``; ``lane_order[k]`` = the
    group-major lane number in ``groups`` of the k-th lane of the passes' concatenated
    results (unpermute_lanes)."""
    if max_lanes < 1:
        raise KPError(-2, "the lattice does not fit device memory even for one lane")
    if width:
        pieces = fold_pieces(groups, max(1, min(width, max_lanes)))
    else:
        start = np.cumsum([0] + [len(g[3]) for g in groups])
        pieces = [[(g[0], g[1], g[2], list(g[3]), list(range(start[i], start[i + 1])))] for i, g in enumerate(groups)]
    desc = sorted(range(len(pieces)), key=lambda i: -pieces[i][0][0])  # stable
    passes, cur, n = [], [], 0
    for i in desc:
        lanes = sum(len(x[3]) for x in pieces[i])
        if cur and n + lanes > max_lanes:
            passes.append(cur)
            cur, n = [], 0
        cur.extend(pieces[i])
        n += lanes
    if cur:
        passes.append(cur)
    passes.reverse()
    # the first pass starts when its highest fold is drawn: if it packs the share's lowest
    # fold with a higher one (e.g. a 1-lane fold-0 piece beside a 4-lane fold-2 piece), the
    # lowest fold's pieces run first on their own (fold 2 is drawn ~65 ms after fold 0 at
    # 9-mers, while packing saves ~10 ms of pass time)
    if passes and len({x[0] for x in passes[0]}) > 1:
        lo = min(x[0] for x in passes[0])
        passes[:1] = [[x for x in passes[0] if x[0] == lo], [x for x in passes[0] if x[0] != lo]]
    # within a pass the fold with the most lanes comes first (lanes 0..): a 1-lane piece laid
    # out before a 5-lane one costs the pass 486 vs 468 ms at 9-mers
    # (profiles/r05/experiments/pack_order.txt); the pieces of one fold stay adjacent, so
    # the library can still cut them into mixed device groups
    for i, pas in enumerate(passes):
        per_fold = {}
        for x in pas:
            per_fold[x[0]] = per_fold.get(x[0], 0) + len(x[3])
        passes[i] = sorted(pas, key=lambda x: (-per_fold[x[0]], x[0]))  # stable within a fold
    lane_order = np.array([lid for pas in passes for x in pas for lid in x[4]], dtype=np.int64)
    return [[tuple(x[:4]) for x in pas] for pas in passes], lane_order


def unpermute_lanes(lane_order, arr):
    """Lane results in the passes' order (plan_passes) back to the groups' own group-major
    lane order."""
    out = np.empty_like(arr)
    out[lane_order] = arr
    return out


_devices = {}
_plans = {}
_cache_lock = threading.Lock()


def get_device(dev, replica=0):
    """The library context of GPU ``dev``; ``replica`` > 0 = another context (its own HIP
    stream) on the same GPU, for a device list that names one GPU more than once."""
    with _cache_lock:
        if (dev, replica) not in _devices:
            _devices[(dev, replica)] = Device(dev)
        return _devices[(dev, replica)]


def get_plan(dev, gen_pat, max_block=0, replica=0):
    key = (dev, gen_pat, max_block, replica)
    with _cache_lock:
        plan = _plans.get(key)
    if plan is None:
        plan = Plan(get_device(dev, replica), gen_pat, max_block)
        with _cache_lock:
            # one resident lattice per device: drop other patterns' buffers first (replicas
            # of the same lattice stay)
            for other in [k for k in _plans if k[0] == dev and k[1:3] != key[1:3]]:
                _plans.pop(other).close()
            _plans[key] = plan
    return plan


def release_all():
    """Free every cached plan's device buffers (the devices stay open)."""
    with _cache_lock:
        for p in _plans.values():
            p.close()
        _plans.clear()


def _shutdown():
    """At interpreter exit, while the library and the HIP runtime are still loaded: plans
    first (a plan's pooled score buffer is freed on its device's stream), then devices.
    Left to garbage collection, module teardown may destroy a device before its plan."""
    try:
        release_all()
        with _cache_lock:
            for d in _devices.values():
                d.close()
            _devices.clear()
    except Exception:
        pass


atexit.register(_shutdown)


def _device_shares(groups, devices, width):
    from .shard import rank_groups
    return [rank_groups(groups, slot, len(devices), width) for slot in range(len(devices))]


def _replicas(devices):
    """Replica index of every slot: how often its GPU was named before (0 for a list of
    distinct GPUs).  A GPU named twice gets two contexts and two host threads: that runs
    the multi-GPU path on one GPU (a rehearsal; the slots share its HBM and bandwidth)."""
    seen = {}
    out = []
    for d in devices:
        out.append(seen.get(d, 0))
        seen[d] = out[-1] + 1
    return out


def prepare_groups(gen_pat, groups, devices=None, max_block=0, itype=np.uint32):
    """Everything ``run_groups`` needs before the counts exist: each GPU's plan (lattice
    tables uploaded) and one allocation for its largest pass.  Only the lane counts of
    ``groups`` matter (folds, alphas and betas may be placeholders), so a caller can run
    this while the host draws the fold split (CV_tools.fold_tables drops the GIL).  ``itype``
    = the counts' width to come (the shares depend on it, shard_width)."""
    devices = list(devices if devices is not None else visible_devices()[:1])
    wg = shard_width(gen_pat, itype, max_block)  # the sweep workgroup's lanes at the counts' width

    errors = []

    def prep(dev, rep, chunk):
        try:
            if chunk:
                plan = get_plan(dev, gen_pat, max_block, replica=rep)
                passes, _ = plan_passes(chunk, pass_cap(chunk, plan.require_lanes(), wg), wg)
                plan.reserve(max(sum(len(g[3]) for g in pas) for pas in passes))
        except Exception as e:  # re-raised in the caller's thread
            errors.append(e)
    threads = [threading.Thread(target=prep, args=(dev, rep, chunk))
               for dev, rep, chunk in zip(devices, _replicas(devices),
                                          _device_shares(groups, devices, wg if len(devices) > 1 else 0))]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    if errors:
        raise errors[0]


PASS_LOG = None  # a list to receive one timing record per pass of run_groups (bench.py)


def run_groups(gen_pat, M, U, groups, devices=None, max_block=0):
    """Run every lane group over the lattice of ``gen_pat`` on the given GPUs.

    ``M``/``U`` are ``[n_kmers, nf]`` counts in k-mer order, or ``M`` is a
    :class:`FoldFeed` (``U`` unused): then every GPU uploads the all-data counts first and
    each fold as it arrives, and runs its passes in fold order, so the first passes start
    before the last folds are drawn.  The lanes (one penalty of one group, group-major)
    are split over the GPUs in equal shares and regrouped by (fold, alpha)
    (``shard.assign_lanes``: whole groups where each fits a workgroup, else contiguous lane
    runs -- the same split the ranks of a torchrun job use),
    each GPU's share packed into memory-sized passes, one host thread per GPU.  Returns
    ``(root_train, root_test, n_leaves)`` arrays over all lanes, group-major.
    """
    devices = list(devices) if devices is not None else visible_devices()[:1]
    reps = _replicas(devices)  # one host thread and one context per slot: a plan is never shared
    if not devices:
        raise KPError(-3, "no GPU visible")
    nd = len(devices)
    # (whole groups of one workgroup's width per device; results go back by shard.unshard)
    width = shard_width(gen_pat, counts_itype(M), max_block) if nd > 1 else 0
    shares = _device_shares(groups, devices, width)
    results = [None] * nd
    errors = []

    feed = M if isinstance(M, FoldFeed) else None

    def work(slot, dev, chunk):
        try:
            outs = []
            if chunk:
                plan = get_plan(dev, gen_pat, max_block, replica=reps[slot])
                if feed is not None:
                    plan.counts_begin(feed.M_all, feed.U_all, feed.nf)
                else:
                    plan.set_counts(M, U)
                # passes in fold order (folds arrive in order), small groups beside a full one
                width = plan.info["lanes_per_workgroup"]
                passes, order = plan_passes(chunk, pass_cap(chunk, plan.require_lanes(), width), width)
                plan.reserve(max(sum(len(g[3]) for g in pas) for pas in passes))  # one allocation
                outs = []
                queued = {}
                if feed is not None:
                    # a feeder thread queues each fold's count table (kp_counts_fold: the
                    # device's count stream) as soon as the fold is drawn, so it fills while
                    # the previous fold's passes run; a pass waits until its folds are queued
                    need = []
                    for pas in passes:
                        need += sorted({g[0] for g in pas if g[0] >= 0} - set(need))
                    queued = {f: threading.Event() for f in need}
                    fed_err = []

                    def feeder():
                        try:
                            for f in need:
                                plan.counts_fold(f, *feed.get(f))
                                queued[f].set()
                        except BaseException as e:  # raised by the pass loop below
                            fed_err.append(e)
                        finally:
                            for ev in queued.values():
                                ev.set()
                    fth = threading.Thread(target=feeder)
                    fth.start()
                try:
                    for pas in passes:
                        t_wait = time.perf_counter()
                        for f in sorted({g[0] for g in pas if g[0] in queued}):
                            queued[f].wait()
                            if fed_err:
                                raise fed_err[0]
                        t_run = time.perf_counter()
                        outs.append(plan.run(pas))
                        if PASS_LOG is not None:  # (slot, lanes, counts wait s, pass start, pass end, stats)
                            PASS_LOG.append((slot, sum(len(g[3]) for g in pas), t_run - t_wait, t_run,
                                             time.perf_counter(), plan.stats() if hasattr(plan, "stats") else {}))
                finally:
                    if feed is not None:
                        fth.join()
            if outs:
                results[slot] = tuple(unpermute_lanes(order, np.concatenate([o[i] for o in outs]))
                                      for i in range(3))
            else:
                results[slot] = (np.zeros(0, np.float32), np.zeros(0, np.float32), np.zeros(0, np.uint64))
        except Exception as e:  # re-raised in the caller's thread
            errors.append(e)

    threads = []
    for slot, dev in enumerate(devices):
        chunk = shares[slot]
        if nd == 1:
            work(slot, dev, chunk)
        else:
            th = threading.Thread(target=work, args=(slot, dev, chunk))
            th.start()
            threads.append(th)
    for th in threads:
        th.join()
    if errors:
        raise errors[0]
    from .shard import unshard
    return tuple(unshard(groups, nd, [r[i] for r in results], width) for i in range(3))


run_groups.prepare = prepare_groups
run_groups.fold_feed = True  # accepts a FoldFeed for M

"""kp_libm.h (the C library's log / log1p restated for the GPU) against the C library of
this process, bit for bit, on the DP's ranges (p and 1 - p in (0, 1], -p for log1p) and
across the whole float64 range, special values included.  The GPU build is checked the
same way on the GPU box (test_gpu_parity.test_device_libm_exact)."""
import ctypes

import numpy as np

from tests.emu import emu as E


def _libm(name):
    libm = ctypes.CDLL("libm.so.6")
    f = getattr(libm, name)
    f.argtypes = [ctypes.c_double]
    f.restype = ctypes.c_double
    return f


def _restated(x, which):
    x = np.ascontiguousarray(x, np.float64)
    y = np.empty_like(x)
    L = E.lib()
    L.emu_libm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    L.emu_libm.restype = None
    L.emu_libm(x.ctypes.data, y.ctypes.data, x.size, which)
    return y


def _inputs(rng, n):
    return np.concatenate([
        rng.uniform(0.0, 1.0, n), 1.0 - rng.uniform(0.0, 1e-3, n), 1.0 + rng.uniform(-0.07, 0.07, n),
        np.exp(rng.uniform(-745.0, 709.0, n)), rng.uniform(0.0, 1e-300, n // 10) * 1e-8,
        np.array([0x7ff8000000000000, 0xfff8000000000000, 0x7ff8000000000123, 0xfffc000000000000],
                 np.uint64).view(np.float64),  # quiet NaNs of both signs, with payloads
        np.array([0.0, -0.0, 1.0, -1.0, -2.5, np.inf, -np.inf, 5e-324, 2.2250738585072014e-308,
                  np.nextafter(1.0, 0), np.nextafter(1.0, 2), 1.0 - 2.0 ** -4, 1.0 + float.fromhex("0x1.09p-4")])])


def _same(a, b):
    return a.view(np.int64) == b.view(np.int64)  # NaNs too: their bits reach the stored scores


def test_libm_log_restatement():
    rng = np.random.RandomState(11)
    x = _inputs(rng, 400_000)
    f = _libm("log")
    want = np.array([f(float(v)) for v in x])
    got = _restated(x, 0)
    bad = ~_same(got, want)
    assert not bad.any(), (x[bad][:5], got[bad][:5], want[bad][:5])


def test_libm_log1p_restatement():
    rng = np.random.RandomState(12)
    x = np.concatenate([-rng.uniform(0.0, 1.0, 400_000), -_inputs(rng, 100_000), _inputs(rng, 100_000),
                        -rng.uniform(0.0, 1e-8, 10_000), np.array([-1.0, -0.2929, -0.29289, 0.41421, 0.41422])])
    f = _libm("log1p")
    want = np.array([f(float(v)) for v in x])
    got = _restated(x, 1)
    bad = ~_same(got, want)
    assert not bad.any(), (x[bad][:5], got[bad][:5], want[bad][:5])


def test_scipy_xlogy_xlog1py_are_libm():
    """The reference's k-mer terms call scipy.special.xlogy / xlog1py (CV module :15-20,
    Fit :26-29); both are x times the C library's log / log1p (not scipy's own cephes
    log1p, which differs in the last bit on ~7 % of inputs), so kp_libm.h restates them too."""
    import scipy.special as sp
    rng = np.random.RandomState(13)
    p = rng.uniform(0.0, 1.0, 200_000)
    u = rng.randint(1, 10**7, 200_000).astype(np.float64)
    assert _same(sp.xlogy(u, p), u * _restated(p, 0)).all()
    assert _same(sp.xlog1py(u, -p), u * _restated(-p, 1)).all()

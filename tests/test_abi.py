"""CPU: the C-ABI library loads, exports every entry point include/ppfit.h
declares with the layout the ctypes binding assumes, and its host-side
np.roots replacement agrees with numpy.  No compute call needs a GPU here."""
import ctypes
import os
import re

import numpy as np
import pytest

from pulseportraiture_amd import _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include",
                      "ppfit.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ppf_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
        assert n in _lib.SIGNATURES, "binding missing for %s" % n


def test_struct_layouts_match():
    lib = _lib.load()
    assert lib.ppf_abi_version() == _lib.ABI_VERSION == 6
    assert lib.ppf_sizeof_fit_desc() == ctypes.sizeof(_lib.FitDesc)
    assert lib.ppf_sizeof_result() == 8 * _lib.RESULT_DOUBLES == 256


def test_workspace_query_and_validation_without_gpu():
    lib = _lib.load()
    d = _lib.FitDesc()
    d.nsub, d.nchan, d.nbin, d.nmodel = 10, 512, 2048, 1
    nb = lib.ppf_fit_workspace_bytes(ctypes.byref(d))
    # X alone is nsub*nchan*nharm complex128 (every sub-int by default)
    assert nb >= 10 * 512 * 1025 * 16
    # x_subints = 2: only two cross-spectrum slots on the fused phase+DM
    # path (X was reserved for every sub-int)
    d.x_subints = 2
    nb2 = lib.ppf_fit_workspace_bytes(ctypes.byref(d))
    assert nb - nb2 == 8 * 512 * 1025 * 16
    # PPF_OPT_NO_X (the caller ruled X out, engine.fit_batch when
    # x_subints() == 0): no slot at all on the fused path
    d.options = _lib.OPT_NO_X
    nb0 = lib.ppf_fit_workspace_bytes(ctypes.byref(d))
    assert nb2 - nb0 == 2 * 512 * 1025 * 16
    d.options = 0
    # off the fused path (nbin 4096: block FFT, moments taken from X) every
    # sub-int streams X whatever x_subints says
    d.nbin = 4096
    nb3 = lib.ppf_fit_workspace_bytes(ctypes.byref(d))
    d.x_subints = 0
    assert lib.ppf_fit_workspace_bytes(ctypes.byref(d)) == nb3
    d.options = _lib.OPT_NO_X          # ignored off the fused path
    assert lib.ppf_fit_workspace_bytes(ctypes.byref(d)) == nb3
    d.options = 0
    # nbin 1000 (nbin/2 = 2^2 5^3) runs on the mixed-radix LDS FFT, nbin/2
    # with a prime factor above 7 (1002 = 2 x 3 x 167, 8186 = 2 x 4093) on
    # its generic-radix stage; odd nbin up to 4095 as a full-length complex
    # transform
    for nb in (1000, 1002, 1022, 8186, 33, 1001, 1023, 4095):
        d.nbin = nb
        assert lib.ppf_fit_workspace_bytes(ctypes.byref(d)) > 0, nb
    # round 6: rows past the LDS transforms fit on the long transforms; with
    # the GetTOAs guess while its profile spectrum fits one workgroup's LDS
    # (nbin up to ~19,000; the brute grid goes to global memory when it does
    # not fit beside it, e.g. ppalign's Ns = nbin); short rows stay refused
    for nb in (16, 31):
        d.nbin = nb
        assert lib.ppf_fit_workspace_bytes(ctypes.byref(d)) == 0, nb
    for nb in (4097, 8191, 8194, 16384, 40000):
        d.nbin = nb
        assert lib.ppf_fit_workspace_bytes(ctypes.byref(d)) > 0, nb
        d.guess, d.guess_Ns = 1, 100
        w100 = lib.ppf_fit_workspace_bytes(ctypes.byref(d))
        assert (w100 > 0) == (nb < 19000), nb
        d.guess_Ns = nb
        wn = lib.ppf_fit_workspace_bytes(ctypes.byref(d))
        assert (wn > 0) == (nb < 19000), nb
        if nb == 16384:                           # grid [nsub][Ns + 8] global
            assert wn - w100 >= d.nsub * (nb + 8) * 8, nb
        d.guess, d.guess_Ns = 0, 100
    d.nbin = (1 << 24) + 2                        # past 2^23 transform points
    assert lib.ppf_fit_workspace_bytes(ctypes.byref(d)) == 0
    # with the GetTOAs guess at nbin 2048 the phase/DM fits take their
    # moments from X by default (every sub-int holds a slot); the fused
    # pass can be forced
    d.nbin, d.x_subints, d.options, d.guess = 2048, 2, 0, 1
    nbg = lib.ppf_fit_workspace_bytes(ctypes.byref(d))
    d.options = _lib.OPT_FUSED_MOM
    assert nbg - lib.ppf_fit_workspace_bytes(ctypes.byref(d)) >= \
        8 * 512 * 1025 * 16
    d.options, d.guess = 0, 0
    # a NULL context is rejected before touching the device
    assert lib.ppf_fit_batch(None, ctypes.byref(d), None) == _lib.PPF_EINVAL
    # get_noise_PS of long rows: any length up to 2^24 transform points
    # (2^25 samples for a power-of-two row), workspace in 256-MB row chunks
    for nb in (1, 2, 33, 8186, 1 << 20, 511 * 1023, 512 * 1000, 1 << 25):
        assert lib.ppf_noise_long_workspace_bytes(3, nb) > 0, nb
    assert lib.ppf_noise_long_workspace_bytes(3, (1 << 25) + 2) == 0
    assert lib.ppf_noise_long_workspace_bytes(1, 0) == 0
    # a power-of-two row needs no chirp buffers: 2 x 2^19 x 16 B per row
    assert lib.ppf_noise_long_workspace_bytes(1, 1 << 20) == \
        2 * (1 << 19) * 16 + 256 * 8
    assert lib.ppf_noise_long(None, 1, 1 << 20, _lib.PPF_F64, None, 4, None,
                              None, 0, None) == _lib.PPF_EINVAL
    # rotation of long rows: Bluestein both ways, any length to 2^23 points
    for nb in (4097, 8194, 16384, 1 << 23):
        assert lib.ppf_rotate_long_workspace_bytes(2, nb, 1) > 0, nb
    assert lib.ppf_rotate_long_workspace_bytes(2, (1 << 24) + 2, 0) == 0
    assert lib.ppf_rotate_long(None, 1, 16384, _lib.PPF_F64, None, None,
                               None, 0, None, 0, None) == _lib.PPF_EINVAL


@pytest.mark.parametrize("seed", range(40))
def test_poly_real_roots_matches_np_roots(seed):
    rng = np.random.default_rng(seed)
    deg = int(rng.integers(1, 7))
    c = rng.normal(size=deg + 1)
    if seed % 5 == 0:               # even polynomial, as in the GM sextic
        c[1::2] = 0.0
    if seed % 7 == 0:
        c[-1] = 0.0                 # trailing zero -> a zero root
    ref = np.roots(c)
    ref = np.sort(np.real(ref[np.imag(ref) == 0.0]))
    got = np.sort(_lib.poly_real_roots(c))
    assert len(got) == len(ref)
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-12)


def test_gauss_portrait_entry_validates_without_gpu():
    """ppf_gauss_portrait_batch rejects a NULL context, and the Python
    wrapper raises evolve_parameter's KeyError for an unknown evolution
    code before touching any device (pplib.py:1082-1084)."""
    import ctypes
    import pytest
    from pulseportraiture_amd import _lib, engine
    lib = _lib.load()
    rc = lib.ppf_gauss_portrait_batch(None, 1, 1, 64, 1, b"000", None, None,
                                      None, None, None, None)
    assert rc != 0
    with pytest.raises(KeyError):
        engine.gauss_portraits("0x0", np.zeros((1, 8)), [0.0], [[1.0]],
                               [1.0], 64)


def test_x_subints_host_rule():
    """engine.x_subints restates k_classify's test: scattering flags, or a
    nonzero initial tau (10**tau when log10_tau)."""
    from pulseportraiture_amd import engine
    flags = np.array([[1, 1, 0, 0, 0], [1, 1, 0, 1, 1], [1, 1, 0, 0, 1],
                      [1, 1, 0, 0, 0]])
    init = np.zeros((4, 5))
    init[3, 3] = 1e-3
    assert engine.x_subints(flags, init, False, 4) == 3
    assert engine.x_subints(flags, init, True, 4) == 4       # 10**0 = 1
    assert engine.x_subints([1, 1, 0, 0, 0], np.zeros((3, 5)), False, 3) == 0


def test_nospace_status_raises():
    """PPF_ST_NOSPACE (a scattering fit without a cross-spectrum slot) is an
    internal error: the host raises instead of writing an all-zero TOA
    (ADVICE round 2)."""
    import pytest
    from pulseportraiture_amd import _lib
    from pulseportraiture_amd.pplib import _raise_status
    with pytest.raises(RuntimeError):
        _raise_status(_lib.ST_NOSPACE | 2)
    _raise_status(2)


def test_box_bounds():
    """scipy bounds lists -> the [5, 2] device box (NaN = unbounded)."""
    import numpy as np
    from pulseportraiture_amd.pplib import _box
    assert _box(None, 5) is None
    assert _box([(None, None)] * 5, 5) is None
    b = _box([(None, None), (None, 40.0), (None, None), (-3.7, None),
              (-10.0, 10.0)], 5)
    assert b.shape == (5, 2)
    np.testing.assert_array_equal(b[1], [np.nan, 40.0])
    np.testing.assert_array_equal(b[3], [-3.7, np.nan])
    np.testing.assert_array_equal(b[4], [-10.0, 10.0])
    # pplib.fit_portrait: only (phase, DM)
    b2 = _box([(-0.5, 0.5), (None, None), (0.0, 1.0)], 2)
    np.testing.assert_array_equal(b2[0], [-0.5, 0.5])
    assert np.isnan(b2[2]).all()


def _tr_problem(rng, t):
    """A random trust-region subproblem: PD, indefinite, badly scaled and
    hard-case (g orthogonal to the lowest eigenvector) instances."""
    n = int(rng.integers(1, 6))
    A = rng.normal(size=(n, n))
    H = A @ A.T
    if t % 3 == 1:
        H -= rng.uniform(0, 3) * np.eye(n)
    if t % 7 == 0:
        D = np.diag(10 ** rng.uniform(-4, 3, size=n))
        H = D @ H @ D
    if t % 11 == 0 and n > 1:
        _, Q = np.linalg.eigh(H)
        g = Q[:, 1:] @ rng.normal(size=n - 1)
    else:
        g = rng.normal(size=n) * 10 ** rng.uniform(-3, 3)
    return H, g, 10 ** rng.uniform(-3, 2)


def test_tr_subproblem_optimality():
    """The Newton solver's exact trust-region step (ppf_device.hpp tr_exact,
    host export) meets the More-Sorensen optimality conditions: |p| <= R,
    (H + l I) p = -g with l >= 0, l (R - |p|) = 0 and H + l I positive
    semi-definite; its model value is no worse than any point of a random
    sample of the ball."""
    rng = np.random.default_rng(0)
    for t in range(3000):
        H, g, R = _tr_problem(rng, t)
        p, hb = _lib.tr_subproblem(H, g, R)
        pn = np.linalg.norm(p)
        assert pn <= R * (1 + 1e-12)
        scale = np.abs(H).max() * max(pn, 1e-300) + np.linalg.norm(g)
        if not hb:
            assert np.linalg.eigvalsh(H)[0] > 0
            assert np.linalg.norm(H @ p + g) <= 1e-8 * scale
            continue
        assert abs(pn - R) <= 1e-9 * R
        lam = -(p @ (H @ p + g)) / (pn * pn)
        assert lam >= -1e-9 * np.abs(H).max()
        assert np.linalg.norm(H @ p + lam * p + g) <= 1e-7 * (scale + lam * pn)
        assert np.linalg.eigvalsh(H + lam * np.eye(len(g)))[0] >= \
            -1e-7 * (np.abs(H).max() + lam)
        if t % 50 == 0:
            v = rng.normal(size=(4000, len(g)))
            v *= (R * rng.uniform(0, 1, size=(4000, 1)) ** (1 / len(g)) /
                  np.linalg.norm(v, axis=1, keepdims=True))
            mv = v @ g + 0.5 * np.einsum("ij,jk,ik->i", v, H, v)
            mp = g @ p + 0.5 * p @ H @ p
            assert mp <= mv.min() + 1e-9 * abs(mv.min())

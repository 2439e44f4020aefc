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
    assert lib.ppf_abi_version() == 1
    assert lib.ppf_sizeof_fit_desc() == ctypes.sizeof(_lib.FitDesc)
    assert lib.ppf_sizeof_result() == 8 * _lib.RESULT_DOUBLES == 256


def test_workspace_query_and_validation_without_gpu():
    lib = _lib.load()
    d = _lib.FitDesc()
    d.nsub, d.nchan, d.nbin, d.nmodel = 10, 512, 2048, 1
    nb = lib.ppf_fit_workspace_bytes(ctypes.byref(d))
    # X alone is nsub*nchan*nharm complex128
    assert nb >= 10 * 512 * 1025 * 16
    d.nbin = 1000   # not a power of two
    assert lib.ppf_fit_workspace_bytes(ctypes.byref(d)) == 0
    # a NULL context is rejected before touching the device
    assert lib.ppf_fit_batch(None, ctypes.byref(d), None) == _lib.PPF_EINVAL


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

"""Host-side logic of the drop-in layer that runs without a GPU: ppalign's
deferred status check (round 6: the status column reaches pinned host memory
behind an event, so the check waits for the fit only) (the reference's exceptions for failed rows, raised
after the iteration's rotate-and-sum is queued; ppalign.py:222-247 through
pptoaslib.py:1068-1079)."""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from pulseportraiture_amd import _lib, ppalign


def _rows(*status):
    # a pending record as _fit_rows queues it: (pinned host copy of the
    # status column, the event behind which it lands; None: already there)
    return (torch.tensor(status, dtype=torch.float64), None)


def test_raise_pending_clean_rows_pass_and_clear():
    R = SimpleNamespace(_dev_inputs={"_pending": [_rows(0, 0, 0)]})
    ppalign.raise_pending(R)
    assert R._dev_inputs["_pending"] == []
    ppalign.raise_pending(R)                 # nothing queued: no-op


@pytest.mark.parametrize("bits,exc", [
    (_lib.ST_NO_ROOT, ValueError),
    (_lib.ST_SINGULAR, np.linalg.LinAlgError),
    (_lib.ST_NOSPACE, RuntimeError),
])
def test_raise_pending_maps_status_to_the_reference_exception(bits, exc):
    R = SimpleNamespace(_dev_inputs={"_pending": [_rows(0, bits | 2, 0)]})
    with pytest.raises(exc):
        ppalign.raise_pending(R)
    assert R._dev_inputs["_pending"] == []   # consumed even when raising


def test_raise_pending_checks_duplicate_channel_rows_too():
    R = SimpleNamespace(_dev_inputs={"_pending": [_rows(0)]},
                        _dup_dev={"_pending": [_rows(_lib.ST_SINGULAR)]})
    with pytest.raises(np.linalg.LinAlgError):
        ppalign.raise_pending(R)


def test_raise_pending_ignores_converged_status_bits():
    # PPF_ST_* low bits (converged / max-iterations) are fit outcomes, not
    # errors: only NO_ROOT, SINGULAR and NOSPACE raise
    R = SimpleNamespace(_dev_inputs={"_pending": [_rows(1, 2, 3)]})
    ppalign.raise_pending(R)


# ---------------------------------------------------------- collectives -----
def test_collective_device_under_nccl_is_the_current_hip_device(monkeypatch):
    """RCCL has no CPU path: the error flag of raise_if_any_failed (and the
    timing max) must live on this rank's HIP device when the caller passes
    none (the archive-sharded get_TOAs did, round 3 ADVICE)."""
    from pulseportraiture_amd import dist
    monkeypatch.setattr(dist, "backend", lambda: "nccl")
    monkeypatch.setattr(dist.torch.cuda, "current_device", lambda: 3)
    assert dist.collective_device() == torch.device("cuda", 3)
    assert dist.collective_device(torch.device("cuda", 1)) == \
        torch.device("cuda", 1)
    monkeypatch.setattr(dist, "backend", lambda: "gloo")
    assert dist.collective_device(torch.device("cuda", 1)) is None


def test_raise_if_any_failed_puts_the_flag_on_the_device(monkeypatch):
    from pulseportraiture_amd import dist
    seen = []
    real_tensor = torch.tensor

    def fake_tensor(v, dtype=None, device=None):
        seen.append(device)
        return real_tensor(v, dtype=dtype)
    monkeypatch.setattr(dist, "is_dist", lambda: True)
    monkeypatch.setattr(dist, "backend", lambda: "nccl")
    monkeypatch.setattr(dist.torch.cuda, "current_device", lambda: 2)
    monkeypatch.setattr(dist.torch, "tensor", fake_tensor)
    monkeypatch.setattr(dist.dist, "all_reduce", lambda t, op=None: None)
    dist.raise_if_any_failed(None)
    with pytest.raises(KeyError):
        dist.raise_if_any_failed(KeyError("x"))
    assert seen == [torch.device("cuda", 2)] * 2


def test_unflat_matches_the_row_table():
    """A one-rank fit's outputs come back as ONE buffer (engine._fit_slice's
    `_flat`: results | scales | scale_errs | channel_snrs | covariance) and
    are cut on the host by pptoas._unflat; the same arrays as the row table
    (_pack / _unpack) the sharded path all-gathers."""
    from pulseportraiture_amd import pptoas
    nsub, nchan = 3, 5
    R = _lib.RESULT_DOUBLES
    sizes = (nsub * R, nsub * nchan, nsub * nchan, nsub * nchan, nsub * 25)
    flat = torch.arange(sum(sizes), dtype=torch.float64)
    views, o = [], 0
    for n in sizes:
        views.append(flat[o:o + n])
        o += n
    res = dict(results=views[0].view(nsub, R),
               scales=views[1].view(nsub, nchan),
               scale_errs=views[2].view(nsub, nchan),
               channel_snrs=views[3].view(nsub, nchan),
               covariance=views[4].view(nsub, 5, 5), _flat=flat)
    a = pptoas._unflat(res, flat.numpy())
    b = pptoas._unpack(pptoas._pack(res).numpy(), nchan)
    for k in ("results", "scales", "scale_errs", "channel_snrs", "covariance"):
        np.testing.assert_array_equal(a[k], b[k])
        np.testing.assert_array_equal(a[k], res[k].numpy())

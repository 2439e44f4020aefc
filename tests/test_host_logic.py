"""Host-side logic of the drop-in layer that runs without a GPU: ppalign's
deferred status check (the reference's exceptions for failed rows, raised
after the iteration's rotate-and-sum is queued; ppalign.py:222-247 through
pptoaslib.py:1068-1079)."""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from pulseportraiture_amd import _lib, ppalign


def _rows(*status):
    return torch.tensor(status, dtype=torch.int64)


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

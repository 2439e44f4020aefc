"""Stand-in for ``past.utils`` (the ``future`` package is not installed here).

``old_div`` is Python-2 division: floor division when both operands are
integers, true division otherwise.  Used only by tests/golden/make_golden.py
when importing the reference to produce golden vectors.
"""
import numbers


def old_div(a, b):
    if isinstance(a, numbers.Integral) and isinstance(b, numbers.Integral):
        return a // b
    return a / b

# Import shim for generating golden vectors only (see tests/golden/make_golden.py).

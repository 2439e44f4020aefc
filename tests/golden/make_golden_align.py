#!/usr/bin/env python
"""Golden vectors for ppalign.align_archives (ppalign.py:65-280), produced by
running the REFERENCE in this container (never on the GPU box).

Same import shims as make_golden.py, plus three stand-ins for what the
reference reaches outside Python: ``load_data`` returns synthetic
DataBunches (the keys of pplib.py:2904-2914), ``subprocess.Popen`` answers
the ``vap -c nchan,nbin`` probe (ppalign.py:111-113), and the PSRCHIVE
archive object at the end (ppalign.py:259-277) is a recorder that captures
the aligned portrait and the channel weights instead of writing a file.

Usage:  python tests/golden/make_golden_align.py
"""
import contextlib
import io
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (imports the reference with the shims)
import numpy as np  # noqa: E402

with contextlib.redirect_stdout(io.StringIO()):
    import ppalign  # noqa: E402


class _Profile:
    def __init__(self, store, ipol, ichan):
        self.store, self.ipol, self.ichan = store, ipol, ichan

    def get_amps(self):
        return self.store[self.ipol, self.ichan]


class _Subint:
    def __init__(self, arch):
        self.arch = arch

    def get_Profile(self, ipol, ichan):
        return _Profile(self.arch.amps, ipol, ichan)

    def set_weight(self, ichan, w):
        self.arch.weights[ichan] = w


class FakeArch:
    """Records what ppalign writes into the output archive."""

    def __init__(self, npol, nchan, nbin):
        self.amps = np.zeros((npol, nchan, nbin))
        self.weights = np.full(nchan, -1.0)
        self.npol = npol
        self.dm = None

    def tscrunch(self):
        pass

    def pscrunch(self):
        pass

    def convert_state(self, state):
        pass

    def set_dispersion_measure(self, dm):
        self.dm = dm

    def get_npol(self):
        return self.npol

    def get_nchan(self):
        return self.amps.shape[1]

    def __iter__(self):
        return iter([_Subint(self)])

    def unload(self, outfile):
        self.outfile = outfile


class _VapPopen:
    def __init__(self, nchan, nbin):
        self.stdout = io.BytesIO(("filename nchan nbin\nguess.fits %d %d\n" %
                                  (nchan, nbin)).encode())


def make_archives(nfile=5, nsub=2, nchan=32, nbin=256, seed=777):
    from pplib import DataBunch
    rng = np.random.default_rng(seed)
    freqs = mg.channel_freqs(nchan)
    phases = mg.pplib.get_bin_centers(nbin)
    files, inputs = {}, {}
    for ifile in range(nfile):
        subints = np.zeros([nsub, 1, nchan, nbin])
        for isub in range(nsub):
            phi = rng.uniform(-0.5, 0.5)
            ddm = rng.normal(3e-4, 2e-4)
            d, model, _ = mg.make_portrait(rng, nchan, nbin, phi, mg.DM0 + ddm,
                                           mg.P0, noise=0.5)
            subints[isub, 0] = d
        weights = np.ones([nsub, nchan])
        if ifile == 2:      # zapped channels in one archive
            weights[:, rng.choice(nchan, 4, replace=False)] = 0.0
        noise = np.array([[mg.pplib.get_noise(subints[i, 0], chans=True)]
                          for i in range(nsub)])
        snrs = np.abs(subints.max(axis=-1)) / noise * 3.0
        wnorm = np.where(weights == 0.0, 0.0, 1.0)
        ok_ichans = [np.compress(wnorm[i], list(range(nchan)))
                     for i in range(nsub)]
        name = "arch%d.fits" % ifile
        files[name] = DataBunch(
            arch=None, DM=mg.DM0, dmc=0, freqs=np.tile(freqs, (nsub, 1)),
            masks=np.einsum("ij,k", wnorm, np.ones(nbin))[:, None],
            nbin=nbin, nchan=nchan, noise_stds=noise, npol=1, nsub=nsub,
            ok_ichans=ok_ichans, ok_isubs=np.arange(nsub), phases=phases,
            prof_SNR=100.0, Ps=np.ones(nsub) * mg.P0, SNRs=snrs,
            subints=subints, weights=weights)
        inputs["f%d_subints" % ifile] = subints[:, 0].astype(np.float32)
        inputs["f%d_weights" % ifile] = weights
        inputs["f%d_snrs" % ifile] = snrs[:, 0]
        inputs["f%d_noise" % ifile] = noise[:, 0]
    # initial guess: archive 0's mean profile, tiled over the channels
    # (make_constant_portrait, notebook cell 17 / SURVEY.md C4)
    prof = mg.f32(files["arch0.fits"].subints[:, 0].mean(axis=(0, 1)))
    guess = np.tile(prof, (nchan, 1))
    arch = FakeArch(1, nchan, nbin)
    files["guess.fits"] = DataBunch(
        arch=arch, DM=0.0, dmc=1, freqs=freqs[None, :],
        masks=np.ones([1, 1, nchan, nbin]), nbin=nbin, nchan=nchan,
        noise_stds=np.ones([1, 1, nchan]), npol=1, nsub=1,
        ok_ichans=[np.arange(nchan)], ok_isubs=np.arange(1), phases=phases,
        prof_SNR=100.0, Ps=np.ones(1) * mg.P0, SNRs=np.ones([1, 1, nchan]),
        subints=guess[None, None], weights=np.ones([1, nchan]))
    inputs["guess"] = guess
    inputs["freqs"] = freqs
    return files, inputs, arch


def run_align(niter=2, nfile=5, nsub=2, nchan=32, nbin=256):
    files, inputs, arch = make_archives(nfile, nsub, nchan, nbin)
    ppalign.load_data = lambda filename, **kw: files[filename]
    ppalign.sub.Popen = lambda *a, **kw: _VapPopen(nchan, nbin)
    datafiles = ["arch%d.fits" % i for i in range(nfile)]
    t0 = time.time()
    with contextlib.redirect_stdout(io.StringIO()):
        ppalign.align_archives(list(datafiles), "guess.fits", fit_dm=True,
                               niter=niter, outfile="aligned.fits",
                               quiet=True)
    dt = time.time() - t0
    out = dict(inputs)
    out.update(nfile=np.int64(nfile), nsub=np.int64(nsub),
               nchan=np.int64(nchan), nbin=np.int64(nbin), niter=np.int64(niter),
               P=np.float64(mg.P0), DM0=np.float64(mg.DM0),
               ref_seconds=np.float64(dt),
               out_aligned=arch.amps[0].copy(), out_weights=arch.weights.copy(),
               out_dm=np.float64(arch.dm))
    return out


def main():
    out = run_align()
    path = os.path.join(HERE, "align.npz")
    np.savez_compressed(path, **out)
    print("wrote %s (%.1f s of reference time)" % (path,
                                                  float(out["ref_seconds"])))


if __name__ == "__main__":
    main()

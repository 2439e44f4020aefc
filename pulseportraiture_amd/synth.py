"""Synthetic wideband sub-integrations for benchmarks and tests.

Mirrors make_fake_pulsar (pplib.py:3302-3499) minus PSRCHIVE, as specified in
SURVEY.md section 8(d): a 3-component Gaussian template portrait (the
example.gmodel of the reference's examples, parameters below), channel
centres linspace(lo + cw/2, lo + bw - cw/2, nchan), each sub-integration the
template rotated by (-phi, -DM) at nu_ref plus white noise.  The data are
generated ON the device (ppf_synth_batch, counter-based RNG keyed by
(seed, sub-integration, channel)), so a shard is reproducible on any rank.
"""
import numpy as np

from . import engine, pplib

P0 = 1.0 / 345.67890123456789      # examples/example.par F0
DM0 = 34.56789                      # examples/example.par DM

# examples/example.gmodel: CODE 000, FREQ 1300 MHz, DC, TAU, ALPHA, then per
# component (loc, m_loc, wid, m_wid, amp, m_amp)
GMODEL_CODE = "000"
GMODEL_NU_REF = 1300.0
GMODEL_ALPHA = -4.0
GMODEL_PARAMS = np.array([
    0.00889801, 0.0,
    0.21925557, -0.00518501, 0.04823579, -2.08031160, 5.13274758, -1.65717015,
    0.23409622, -0.00271530, 0.01573809, 1.61520300, 9.46117549, -2.07617616,
    0.25844309, 0.00288377, 0.02348129, -3.30015260, 2.71065613, -0.90424701,
])


def write_gmodel(path, name="PSR_1234-5678"):
    """The example template as a .gmodel file (the ppgauss format
    read_model parses, pplib.py:2990-3026)."""
    p = GMODEL_PARAMS
    lines = ["MODEL   %s" % name, "CODE    %s" % GMODEL_CODE,
             "FREQ    %.5f" % GMODEL_NU_REF, "DC      %.8f 1" % p[0],
             "TAU     %.8f 1" % p[1], "ALPHA   %.3f      0" % GMODEL_ALPHA]
    for i in range((len(p) - 2) // 6):
        c = p[2 + 6 * i:8 + 6 * i]
        lines.append("COMP%02d  " % (i + 1) +
                     "  ".join("%.8f 1" % v for v in c))
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    return path


def channel_freqs(nchan, lo=1100.0, bw=800.0):
    cw = bw / nchan
    return np.linspace(lo + cw / 2, lo + bw - cw / 2, nchan)


def template(nchan, nbin, lo=1100.0, bw=800.0):
    """(model [nchan, nbin] float64, freqs [nchan]) of the example template."""
    freqs = channel_freqs(nchan, lo, bw)
    model = pplib.gen_gaussian_portrait(GMODEL_CODE, GMODEL_PARAMS,
                                        GMODEL_ALPHA,
                                        pplib.get_bin_centers(nbin), freqs,
                                        GMODEL_NU_REF)
    return model, freqs


def truths(nsub, seed, first=0):
    """Per-sub-integration (phi, DM) drawn as in SURVEY.md 8(d), keyed by the
    global sub-integration index so shards are reproducible."""
    phi = np.empty(nsub)
    dm = np.empty(nsub)
    for i in range(nsub):
        rng = np.random.default_rng(seed + first + i)
        phi[i] = rng.uniform(-0.5, 0.5)
        dm[i] = DM0 + rng.normal(3e-4, 2e-4)
    return phi, dm


def scattered(model, freqs, tau, alpha, nu_tau):
    """The portrait convolved with the one-sided exponential scattering kernel
    of the fit model: rfft(model_n) x B_nk, B_nk = 1 / (1 + 2 pi i k tau_n),
    tau_n = tau (nu_n / nu_tau)^alpha [rot] (pplib.py:4212-4260)."""
    nbin = model.shape[-1]
    k = np.arange(nbin // 2 + 1)
    taus = tau * (np.asarray(freqs) / nu_tau) ** alpha
    B = 1.0 / (1.0 + 2j * np.pi * np.outer(taus, k))
    return np.fft.irfft(np.fft.rfft(model, axis=-1) * B, n=nbin, axis=-1)


def make_batch(nsub, nchan, nbin, seed=20250217, first=0, noise=1.5,
               nu_ref=1500.0, dtype="float32", dev=None, lo=1100.0, bw=800.0,
               tau=0.0, alpha=GMODEL_ALPHA, nu_tau=None):
    """Device batch: dict(data [nsub,nchan,nbin] device tensor, model, freqs,
    P, phi_true, DM_true[, tau_true, alpha_true, nu_tau]).  tau > 0 injects
    scattering (tau [rot] at nu_tau, default nu_ref) into every sub-int; the
    returned `model` is the unscattered template the fit starts from."""
    import torch
    model, freqs = template(nchan, nbin, lo, bw)
    phi, dm = truths(nsub, seed, first)
    P = np.full(nsub, P0)
    src = model
    if tau > 0.0:
        nu_tau = nu_ref if nu_tau is None else nu_tau
        src = scattered(model, freqs, tau, alpha, nu_tau)
    data = engine.synth(src, freqs, phi, dm, P, nu_ref, noise, seed,
                        torch.float32 if dtype == "float32" else torch.float64,
                        dev=dev, first=first)
    out = dict(data=data, model=model, freqs=freqs, P=P, phi_true=phi,
               DM_true=dm, nu_ref=nu_ref)
    if tau > 0.0:
        out.update(tau_true=tau, alpha_true=alpha, nu_tau=nu_tau)
    return out

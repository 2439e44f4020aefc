"""Full-shape golden cases (tests/golden/full.npz, oracle_c5.npz): inputs
rebuilt from their stored parameters by tests/golden/full_inputs.py and
verified against the stored SHA-256 before any comparison."""
import os
import sys

import numpy as np

import goldens as G

sys.path.insert(0, G.GOLDEN)
import full_inputs as FI  # noqa: E402
import synth_np as S  # noqa: E402


def case(kind, name, fname="full.npz"):
    return G.load_case(fname, "%s_%s" % (kind, name))


def _conf(table, name):
    for c in table:
        if c["name"] == name:
            return c
    raise KeyError(name)


def fit_case(name):
    """(golden case, data f32 [nchan, nbin], model, freqs)."""
    c = case("fit", name)
    conf = _conf(FI.FITS, name)
    if conf.get("narrow"):
        FI.write_narrow()
    data, model, freqs, P, truth, init, nu_fit = FI.fit_inputs(conf)
    got = S.sha(data.astype(np.float32), model.astype(np.float32))
    assert got == str(c["sha"]), "rebuilt inputs of %s differ" % name
    return c, data.astype(np.float32), model, freqs


def c5_case(name):
    c = case("c5", name, "oracle_c5.npz")
    conf = _conf(FI.C5, name)
    data, model, freqs, P, truth, init, nu_fit = FI.c5_inputs(conf)
    got = S.sha(data.astype(np.float32), model.astype(np.float32))
    assert got == str(c["sha"]), "rebuilt inputs of %s differ" % name
    return c, data.astype(np.float32), model, freqs, P


def toa_conf(name):
    """The full_inputs.TOAS entry of a get_TOAs case."""
    return _conf(FI.TOAS, name)


def toa_case(name):
    """(golden case, [per-archive dict(subints f32 [nsub, nchan, nbin],
    weights, dfs, epochs, parangles, noise, snrs)], freqs, template path)."""
    c = case("toas", name)
    conf = toa_conf(name)
    gm = FI.toa_gmodel(conf)
    files, freqs = FI.toa_inputs(conf)
    out = []
    for f, fi in enumerate(files):
        sub = fi["subints"].astype(np.float32)
        assert S.sha(sub) == str(c["sha"][f]), \
            "rebuilt inputs of %s archive %d differ" % (name, f)
        np.testing.assert_array_equal(fi["weights"], c["f%d_weights" % f])
        out.append(dict(subints=sub, weights=fi["weights"], dfs=fi["dfs"],
                        epochs=fi["epochs"], parangles=fi["parangles"],
                        noise=c["f%d_noise" % f], snrs=c["f%d_snrs" % f]))
    return c, out, freqs, gm


def toa_archive_fields(name, fi, freqs):
    """load_data DataBunch fields of one rebuilt archive (as the golden
    generator handed them to the reference), minus epochs / phases."""
    return FI.archive_fields(toa_conf(name), fi, freqs, fi["noise"],
                             fi["snrs"])


def align_case(name):
    """(golden case, archives, model_data) as handed to the reference's
    align_archives by make_golden_full.py."""
    c = case("align", name)
    conf = _conf(FI.ALIGNS, name)
    arch, guess, freqs, tfreqs = FI.align_inputs(conf)
    sha = S.sha(np.stack([a["subints"] for a in arch]).astype(np.float32),
                guess)
    assert sha == str(c["sha"]), "rebuilt inputs of %s differ" % name
    nsub, nbin = int(c["nsub"]), int(c["nbin"])
    nchan = int(c["nchan"])
    archives = []
    for f, a in enumerate(arch):
        w = a["weights"]
        wn = np.where(w == 0.0, 0.0, 1.0)
        archives.append(G.Bunch(
            DM=float(c["DM0"]), dmc=0, freqs=np.tile(freqs, (nsub, 1)),
            masks=np.einsum("ij,k", wn, np.ones(nbin))[:, None], nbin=nbin,
            nchan=nchan, noise_stds=c["f%d_noise" % f][:, None], npol=1,
            nsub=nsub, ok_ichans=[np.compress(wn[j], list(range(nchan)))
                                  for j in range(nsub)],
            ok_isubs=np.arange(nsub), prof_SNR=100.0,
            Ps=np.ones(nsub) * float(c["P"]), SNRs=c["f%d_snrs" % f][:, None],
            subints=a["subints"].astype(np.float32).astype(np.float64)[:, None],
            weights=w, state="Intensity"))
    tn = len(tfreqs)
    model_data = G.Bunch(
        DM=0.0, dmc=1, freqs=tfreqs[None, :], masks=np.ones([1, 1, tn, nbin]),
        nbin=nbin, nchan=tn, noise_stds=np.ones([1, 1, tn]), npol=1, nsub=1,
        ok_ichans=[np.arange(tn)], ok_isubs=np.arange(1), prof_SNR=100.0,
        Ps=np.ones(1) * float(c["P"]), SNRs=np.ones([1, 1, tn]),
        subints=guess[None, None], weights=np.ones([1, tn]), arch=None,
        state="Intensity")
    return c, archives, model_data


def align_synthetic(nchan, nbin, nsub, nfile, seed, noise=0.5):
    """(archives, model_data) of a synthetic align run (no golden: the
    oracle's align_archives is the checker), built like align_case's with
    full_inputs.align_inputs; noise stds at the synthesis level and unit
    S/N weights."""
    conf = dict(nchan=nchan, nbin=nbin, nsub=nsub, nfile=nfile, seed=seed,
                noise=noise)
    arch, guess, freqs, tfreqs = FI.align_inputs(conf)
    archives = []
    for a in arch:
        w = a["weights"]
        wn = np.where(w == 0.0, 0.0, 1.0)
        archives.append(G.Bunch(
            DM=float(S.DM0), dmc=0, freqs=np.tile(freqs, (nsub, 1)),
            masks=np.einsum("ij,k", wn, np.ones(nbin))[:, None], nbin=nbin,
            nchan=nchan, noise_stds=np.full((nsub, 1, nchan), noise), npol=1,
            nsub=nsub, ok_ichans=[np.compress(wn[j], list(range(nchan)))
                                  for j in range(nsub)],
            ok_isubs=np.arange(nsub), prof_SNR=100.0,
            Ps=np.ones(nsub) * float(S.P0), SNRs=np.ones((nsub, 1, nchan)),
            subints=a["subints"].astype(np.float32).astype(np.float64)[:, None],
            weights=w, state="Intensity"))
    tn = len(tfreqs)
    model_data = G.Bunch(
        DM=0.0, dmc=1, freqs=tfreqs[None, :], masks=np.ones([1, 1, tn, nbin]),
        nbin=nbin, nchan=tn, noise_stds=np.ones([1, 1, tn]), npol=1, nsub=1,
        ok_ichans=[np.arange(tn)], ok_isubs=np.arange(1), prof_SNR=100.0,
        Ps=np.ones(1) * float(S.P0), SNRs=np.ones([1, 1, tn]),
        subints=guess[None, None], weights=np.ones([1, tn]), arch=None,
        state="Intensity")
    return archives, model_data

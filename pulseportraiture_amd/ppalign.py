"""Drop-in mirror of PulsePortraiture's ``ppalign.align_archives``
(ppalign.py:65-280): iterative phase/DM alignment and weighted averaging of
homogeneous archives into a template portrait (BASELINE.json configs[3]).

Per iteration the reference loops over archives and sub-integrations with
one ``fit_portrait_full`` and one ``rotate_data`` each (ppalign.py:118-247).
Here every usable sub-integration of every archive goes into ONE batched
device fit (``ppf_fit_batch``: the ``fit_phase_shift(Ns=nbin)`` guess on the
dedispersed weighted mean profile, the phase+DM wideband fit, ν₀, scales),
and the weighted sum of the rotated sub-integrations is ONE device call
(``ppf_align_accum``: rotation and accumulation in the frequency domain, a
fixed summation order).  The data are loaded once and stay resident in HBM
across iterations (the reference re-reads every archive every iteration).

Multi-GPU: pass ``comm=True`` inside a ``torch.distributed`` job and give
each rank its share of ``metafile``; the aligned portrait and the channel
weights are summed across ranks with one all-reduce per iteration (RCCL over
xGMI), the only exchange the algorithm has.

Archive I/O stays on PSRCHIVE (``pptoas.load_data``, host side); the output
archive is written through the template archive object exactly as
ppalign.py:259-277 does when one is attached (``model_data.arch``).
"""
import numpy as np
import torch

from . import _lib, engine
from . import pptoas as _pptoas
from .pplib import (DataBunch, Dconst, fit_phase_shift, gaussian_profile,
                    get_noise, guess_fit_freq, rotate_data)

rm_baseline = _pptoas.rm_baseline       # ppalign.py imports it from pptoas


def normalize_portrait(port, method="rms", weights=None, return_norms=False):
    """pplib.py:2553-2600."""
    if method not in ("mean", "max", "prof", "rms", "abs"):
        print("Unknown method for normalize_portrait(...), '%s'." % method)
        return None
    port = np.asarray(port, dtype=np.float64)
    norm_port = np.zeros(port.shape)
    norm_vals = np.ones(len(port))
    if method == "prof":
        good = np.where(port.sum(axis=1) != 0.0)[0]
        w = np.ones(len(good)) if weights is None else weights[good]
        mean_prof = np.average(port[good], axis=0, weights=w)
    for ichan in range(len(port)):
        if port[ichan].any():
            if method == "mean":
                norm = port[ichan].mean()
            elif method == "max":
                norm = port[ichan].max()
            elif method == "prof":
                norm = fit_phase_shift(port[ichan], mean_prof).scale
            elif method == "rms":
                norm = get_noise(port[ichan])
            else:
                norm = (port[ichan] ** 2.0).sum() ** 0.5
            norm_port[ichan] = port[ichan] / norm
            norm_vals[ichan] = norm
    if return_norms:
        return norm_port, norm_vals
    return norm_port


def _load(name, state, tscrunch, pscrunch, quiet):
    return _pptoas.load_data(name, state=state, dedisperse=False,
                             tscrunch=tscrunch, pscrunch=pscrunch,
                             fscrunch=False, rm_baseline=rm_baseline,
                             flux_prof=False, refresh_arch=False,
                             return_arch=False, quiet=quiet)


def _usable(data, name, model_data, SNR_cutoff, quiet):
    """The reference's per-archive skip tests (ppalign.py:155-185); returns
    False to skip.  Channels with a NaN S/N are dropped in place."""
    if data.nbin != model_data.nbin:
        if not quiet:
            print("%s: %d != %d phase bins.  Skipping it." %
                  (name, data.nbin, model_data.nbin))
        return False
    if data.prof_SNR < SNR_cutoff:
        if not quiet:
            print("%s: %d < %d S/N cutoff.  Skipping it." %
                  (name, data.prof_SNR, SNR_cutoff))
        return False
    if np.isnan(data.prof_SNR):
        print("Profile has nan SNR, must skip")
        return False
    nnan = len(data.SNRs[np.isnan(data.SNRs)])
    if nnan > 10:
        print("More than 10 frequency channels with nan SNR")
        return False
    if nnan:
        print("This file has %s frequency channels with a nan SNR" % nnan)
        print(name)
        for isub in data.ok_isubs:
            for ipol in range(data.npol):
                oc = np.array(data.ok_ichans[isub])
                data.ok_ichans[isub] = oc[~np.isnan(data.SNRs[isub, ipol][oc])]
    return True


def _channel_map(data, isub, model_data, same_freqs):
    """(ichans, model_ichans) of ppalign.py:192-207."""
    if same_freqs:
        ichans = np.intersect1d(data.ok_ichans[isub], model_data.ok_ichans[0])
        return ichans, ichans
    ichans = np.asarray(data.ok_ichans[isub])
    mok = np.asarray(model_data.ok_ichans[0])
    mch = np.array([mok[np.argmin(abs(model_data.freqs[0][mok] -
                                      data.freqs[isub, ic]))]
                    for ic in ichans], dtype=int)
    return ichans, mch


class _Rows(object):
    """Every usable sub-integration of every archive, device-resident.

    The accumulation layout is MODEL channel order (row s, channel m = the
    data channel mapped onto model channel m): numpy's fancy-index "+=" of
    ppalign.py:244-247 keeps the LAST of several data channels mapped onto
    one model channel, so only that one is placed there.  The fit, however,
    runs over the full ichans list (ppalign.py:198-227: the guess profile,
    nu_fit and fit_portrait_full all see every data channel, duplicates
    included): rows without duplicate model channels are fitted in model
    order against the shared template; rows with duplicates get a second,
    data-order ("slot") layout whose model rows are gathered from the
    template by model channel (`dup_*` below)."""

    def __init__(self, archives, model_data, npol, dev):
        nchan, nbin = model_data.nchan, model_data.nbin
        rows, meta, dup = [], [], []
        exact = True                 # every amplitude survives a float32 trip
        for data in archives:
            try:
                fd = data.freqs - model_data.freqs
                same = fd.min() == fd.max() == 0.0
            except Exception:
                same = False
            DM_guess = data.DM * np.logical_not(data.dmc)
            for isub in data.ok_isubs:
                ichans, mch = _channel_map(data, isub, model_data, same)
                if len(ichans) == 0:
                    continue
                last = {}
                for i, m in enumerate(mch):
                    last[int(m)] = i
                sel = np.array(sorted(last.values()), dtype=int)
                ich, mchl = ichans[sel], mch[sel]
                x = np.zeros((npol, nchan, nbin))
                for ipol in range(npol):
                    x[ipol, mchl] = data.subints[isub, ipol, ich]
                    if exact:
                        v = np.asarray(data.subints[isub, ipol, ichans])
                        exact = np.array_equal(
                            v.astype(np.float32).astype(np.float64), v)
                freqs = np.ones(nchan) * np.nan
                freqs[mchl] = data.freqs[isub, ich]
                m = dict(mask=np.zeros(nchan, np.uint8), freqs=freqs,
                         P=float(data.Ps[isub]), DM_guess=float(DM_guess),
                         DM=float(data.DM), errs=np.ones(nchan),
                         gw=np.zeros(nchan), nchanx=len(ichans),
                         dup=len(sel) < len(ichans))
                m["mask"][mchl] = 1
                m["errs"][mchl] = data.noise_stds[isub, 0, ich]
                m["gw"][mchl] = data.weights[isub, ich]
                # guess_fit_freq over the full ichans (ppalign.py:214)
                m["nu_fit"] = guess_fit_freq(data.freqs[isub, ichans],
                                             data.SNRs[isub, 0, ichans])
                if m["dup"] and len(ichans) > 1:
                    dup.append(dict(
                        row=len(rows), mch=np.asarray(mch, dtype=int),
                        last=sel, x=np.asarray(data.subints[isub, 0, ichans],
                                               dtype=np.float64),
                        freqs=np.asarray(data.freqs[isub, ichans], float),
                        errs=np.asarray(data.noise_stds[isub, 0, ichans],
                                        float),
                        gw=np.asarray(data.weights[isub, ichans], float)))
                rows.append(x)
                meta.append(m)
        self.n = len(rows)
        self.meta = meta
        # float32 amplitudes (PSRCHIVE's type) unless some value would not
        # survive the round trip (e.g. after rm_baseline): then float64
        self.dtype = np.float32 if exact else np.float64
        if self.n:
            self.data = torch.as_tensor(
                np.stack(rows).astype(self.dtype)).to(dev)  # [S, npol, nchan, nbin]
        fill = np.nanmean([np.nanmean(m["freqs"]) for m in meta]) if meta else 1.0
        self.freqs = np.array([np.where(np.isnan(m["freqs"]), fill, m["freqs"])
                               for m in meta])
        self.mask = np.array([m["mask"] for m in meta])
        self.errs = np.array([m["errs"] for m in meta])
        self.gw = np.array([m["gw"] for m in meta])
        self.P = np.array([m["P"] for m in meta])
        self.DM_guess = np.array([m["DM_guess"] for m in meta])
        self.nu_fit = np.array([m["nu_fit"] for m in meta])
        self.nchanx = np.array([m["nchanx"] for m in meta])
        self.dup = np.array([m["dup"] for m in meta], dtype=bool)
        self.dup_rows = dup
        self._dup_dev = None
        if dup:
            self._dup_layout(dev, fill)

    def _dup_layout(self, dev, fill):
        """Slot-order inputs of the rows with duplicate model channels:
        slot j of row d = data channel ichans[j] (model channel mch[j]),
        padded with masked slots to the longest ichans.  Rows with the same
        mch list share one gathered model (index `gidx`)."""
        D = self.dup_rows
        nchf = max(len(d["mch"]) for d in D)
        nbin = D[0]["x"].shape[1]
        x = np.zeros((len(D), nchf, nbin))
        mask = np.zeros((len(D), nchf), np.uint8)
        freqs = np.full((len(D), nchf), fill)
        errs = np.ones((len(D), nchf))
        gw = np.zeros((len(D), nchf))
        groups, gidx, midx = {}, [], []
        for i, d in enumerate(D):
            n = len(d["mch"])
            x[i, :n], mask[i, :n] = d["x"], 1
            freqs[i, :n], errs[i, :n], gw[i, :n] = d["freqs"], d["errs"],                 d["gw"]
            key = tuple(d["mch"])
            if key not in groups:
                groups[key] = len(gidx)
                gidx.append(np.pad(d["mch"], (0, nchf - n)))
            midx.append(groups[key])
        f64 = torch.float64
        rows = [d["row"] for d in D]
        init = np.zeros((len(D), 5))
        init[:, 1] = self.DM_guess[rows]
        self._dup_dev = dict(
            x=torch.as_tensor(x.astype(self.dtype)).to(dev),
            mask=torch.as_tensor(mask, device=dev),
            freqs=torch.as_tensor(freqs, dtype=f64, device=dev),
            errs=torch.as_tensor(errs, dtype=f64, device=dev),
            gw=torch.as_tensor(gw, dtype=f64, device=dev),
            P=torch.as_tensor(self.P[rows], dtype=f64, device=dev),
            DM=torch.as_tensor(self.DM_guess[rows], dtype=f64, device=dev),
            init=torch.as_tensor(init, dtype=f64, device=dev),
            nu_fits=torch.as_tensor(np.repeat(self.nu_fit[rows, None], 3,
                                              axis=1), dtype=f64, device=dev),
            nu_outs=torch.full((len(D), 3), float("nan"), dtype=f64,
                               device=dev),
            gidx=torch.as_tensor(np.array(gidx), dtype=torch.int64,
                                 device=dev),
            midx=np.array(midx, dtype=np.int32))


def _fit_rows(rows, model, mi, dc, fit_dm, nbin, dev):
    """One batched ppf_fit_batch of `rows` (guess + phase[/DM] fit), the
    reference's exceptions raised for failed sub-ints."""
    # the flags stay resident with the rows' other inputs (a host list would
    # be staged and copied in every iteration)
    key = "flags%d" % int(bool(fit_dm))
    if key not in dc:
        dc[key] = torch.tensor([1, int(bool(fit_dm)), 0, 0, 0],
                               dtype=torch.int32, device=dev)
    flags = dc[key]
    # no scattering and a zero initial tau (init holds only the DM): no
    # sub-int streams the cross spectrum -- known on the host, so fit_batch
    # need not read the device-resident init back to count them
    res = engine.fit_batch(
        rows, model, dc["freqs"], dc["P"], dc["init"], flags,
        nu_fits=dc["nu_fits"], nu_outs=dc["nu_outs"], errs=dc["errs"],
        chan_mask=dc["mask"], model_index=mi, log10_tau=False, is_toa=True,
        guess=True, guess_weights=dc["gw"], guess_DM=dc["DM"],
        guess_Ns=nbin, dev=dev, guess_ref=1,   # ppalign.py:214-219: at nu_fit
        n_x=0, spin_wait=True)
    I = _lib.RESULT_INDEX
    r = res["results"]
    dc["last_results"] = r               # (diagnostics: bench.py --fit align)
    # the status bits are checked by raise_pending() once the iteration's
    # rotate-and-sum is queued.  They travel to pinned host memory as soon
    # as the fit has written them, behind an event, so the check waits for
    # the fit only -- not for the rotate-and-sum queued after it, during
    # which the host queues the next iteration (round 6: a .cpu() here
    # waited for the whole queue and left the device idle while the host
    # set up the next iteration, ~0.3 ms of a 3-ms C4 iteration)
    st = r[:, I["status"]]
    hs = torch.empty(st.shape, dtype=st.dtype, pin_memory=True)
    hs.copy_(st, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    dc.setdefault("_pending", []).append((hs, ev))
    # phases and weights in one launch (ppf_align_phases; the elementwise
    # torch form was a dozen launches and Python round trips per iteration
    # while the device waited for them)
    ph, wt = engine.align_phases(r, dc["freqs"], dc["P"], dc["mask"],
                                 res["scales"], dc["errs"], dev)
    return ph, wt


def raise_pending(R):
    """The reference's exceptions for the failed rows of the iteration's
    fits (pptoaslib.py:1068-1079): reads back the status bits _fit_rows
    queued, after the caller has queued the work that uses the fits."""
    from .pplib import _raise_status
    for dc in (R.__dict__.get("_dev_inputs"), getattr(R, "_dup_dev", None)):
        if not dc or not dc.get("_pending"):
            continue
        sts, dc["_pending"] = dc["_pending"], []
        for hs, ev in sts:
            if ev is not None:           # (None: host-resident already)
                ev.synchronize()
            st = hs.numpy().astype(np.int64)
            bad = np.where(st & (_lib.ST_NO_ROOT | _lib.ST_SINGULAR |
                                 _lib.ST_NOSPACE))[0]
            if len(bad):
                _raise_status(int(st[bad[0]]))


def _fit_and_weights(R, model_port, fit_dm, nbin, dev):
    """One batched fit of every row against the current template: the
    per-row rotation phases and weights of ppalign.py:222-247 (model
    channel order)."""
    S = R.n
    nchan = model_port.shape[0]
    f64 = torch.float64
    dup = getattr(R, "dup", np.zeros(S, dtype=bool))
    multi = np.where((R.nchanx > 1) & ~dup)[0]
    # the rows' constant inputs stay resident across iterations
    dc = R.__dict__.setdefault("_dev_inputs", {})
    if dc.get("multi") is None or not np.array_equal(dc["multi"], multi):
        dc.clear()
        dc["multi"] = multi
        dc["freqs"] = torch.as_tensor(R.freqs[multi], dtype=f64, device=dev)
        dc["P"] = torch.as_tensor(R.P[multi], dtype=f64, device=dev)
        dc["errs"] = torch.as_tensor(R.errs[multi], dtype=f64, device=dev)
        dc["mask"] = torch.as_tensor(R.mask[multi], dtype=torch.uint8,
                                     device=dev)
        dc["gw"] = torch.as_tensor(R.gw[multi], dtype=f64, device=dev)
        dc["DM"] = torch.as_tensor(R.DM_guess[multi], dtype=f64, device=dev)
        init = np.zeros((len(multi), 5))
        init[:, 1] = R.DM_guess[multi]
        dc["init"] = torch.as_tensor(init, dtype=f64, device=dev)
        dc["nu_fits"] = torch.as_tensor(
            np.repeat(R.nu_fit[multi, None], 3, axis=1), dtype=f64,
            device=dev)
        dc["nu_outs"] = torch.full((len(multi), 3), float("nan"), dtype=f64,
                                   device=dev)
    # every row fitted in the one batch (the usual case): its phases and
    # weights are the iteration's, with no zero-filled tensors to place them
    # in (two fill launches fewer per iteration)
    phases = weights = None
    if len(multi):
        rows = R.data[:, 0] if len(multi) == S else \
            R.data[torch.as_tensor(multi, device=dev), 0]
        ph, wt = _fit_rows(rows, model_port, None, dc, fit_dm, nbin, dev)
        if len(multi) == S:
            phases, weights = ph, wt
        else:
            phases = torch.zeros((S, nchan), dtype=f64, device=dev)
            weights = torch.zeros((S, nchan), dtype=f64, device=dev)
            mi = torch.as_tensor(multi, device=dev)
            phases[mi] = ph
            weights[mi] = wt
    if phases is None:
        phases = torch.zeros((S, nchan), dtype=f64, device=dev)
        weights = torch.zeros((S, nchan), dtype=f64, device=dev)
    if getattr(R, "_dup_dev", None) is not None:
        # rows with duplicate model channels: fit in slot order against the
        # gathered template rows, then place each model channel's LAST slot
        dd = R._dup_dev
        mp = torch.as_tensor(np.asarray(model_port) if not isinstance(
            model_port, torch.Tensor) else model_port, dtype=f64, device=dev)
        models = mp[dd["gidx"]]                       # [G, nchf, nbin]
        ph, wt = _fit_rows(dd["x"], models, dd["midx"], dd, fit_dm, nbin,
                           dev)
        for i, d in enumerate(R.dup_rows):
            s, last = d["row"], torch.as_tensor(d["last"], device=dev)
            m = torch.as_tensor(d["mch"][d["last"]], device=dev)
            phases[s, m] = ph[i, last]
            weights[s, m] = wt[i, last]
    for s in np.where(R.nchanx == 1)[0]:      # 1-channel hack (ppalign.py:231-236)
        m = int(np.where(R.mask[s])[0][0])
        x = R.data[s, 0, m].double().cpu().numpy()
        mrow = model_port[m]
        if isinstance(mrow, torch.Tensor):
            mrow = mrow.cpu().numpy()
        fr = fit_phase_shift(x, mrow, R.errs[s, m], Ns=nbin)
        phases[s, m] = fr.phase          # DM = data.DM at nu_ref = freqs[0]: 0
        weights[s, m] = fr.scale / R.errs[s, m] ** 2
    return phases, weights


def align_archives(metafile, initial_guess, fit_dm=True, tscrunch=False,
                   pscrunch=True, SNR_cutoff=0.0, outfile=None, norm=None,
                   rot_phase=0.0, place=None, niter=1, quiet=False,
                   comm=False, dev=None):
    """ppalign.py:65-280.  Returns a DataBunch(port=[npol, nchan, nbin]
    aligned portrait, total_weights=[nchan, nbin], nit=niter) and, like the
    reference, writes ``outfile`` through ``model_data.arch`` when the
    template archive object is attached."""
    if isinstance(metafile, str):
        datafiles = [l[:-1] for l in open(metafile, "r").readlines()]
        if outfile is None:
            outfile = metafile + ".algnd.fits"
    else:
        datafiles = list(metafile)
    state, npol = ("Intensity", 1) if pscrunch else ("Stokes", 4)
    try:
        model_data = _pptoas.load_data(
            initial_guess, state=state, dedisperse=True, dededisperse=False,
            tscrunch=True, pscrunch=pscrunch, fscrunch=False,
            rm_baseline=True, flux_prof=False, refresh_arch=True,
            return_arch=True, quiet=quiet)
    except IndexError:
        print("%s: has npol = 1; need npol == 4." % initial_guess)
        raise SystemExit
    nchan, nbin = model_data.nchan, model_data.nbin
    model_port = np.asarray((model_data.masks * model_data.subints)[0, 0],
                            dtype=np.float64)
    dev = engine.device(dev)
    # archives are read once and kept resident (the reference re-reads them
    # every iteration; the skip tests give the same outcome each time)
    from . import dist as _dist
    archives, err = [], None
    try:
        for name in datafiles:
            try:
                data = _load(name, state, tscrunch, pscrunch, quiet)
            except RuntimeError:
                if not quiet:
                    print("%s: cannot load_data().  Skipping it." % name)
                continue
            except IndexError:
                if not quiet:
                    print("%s: has npol = 1.  Skipping it." % name)
                continue
            if _usable(data, name, model_data, SNR_cutoff, quiet):
                archives.append(data)
        R = _Rows(archives, model_data, npol, dev)
    except Exception as exc:
        if not comm:
            raise
        err = exc
    if comm:
        _dist.raise_if_any_failed(err, dev)
    count = 1
    while niter:
        if not quiet:
            print("Doing iteration %d..." % count)
        out = torch.zeros((npol, nchan, nbin), dtype=torch.float64, device=dev)
        wsum = torch.zeros(nchan, dtype=torch.float64, device=dev)
        err = None
        try:
            if R.n:
                phases, weights = _fit_and_weights(R, model_port, fit_dm,
                                                   nbin, dev)
                for ipol in range(npol):
                    # the weight sum once (ipol 0); the other pols' into a
                    # scratch that is dropped
                    w = wsum if ipol == 0 else torch.zeros_like(wsum)
                    engine.align_accum(R.data[:, ipol], phases, weights,
                                       out[ipol], w, dev=dev)
                raise_pending(R)
        except Exception as exc:        # raised on every rank, below
            if not comm:
                raise
            err = exc
        if comm:
            # a failed rank must not leave the others blocked in the
            # all-reduce: agree on success first
            _dist.raise_if_any_failed(err, dev)
            _dist.allreduce_sum_(out, wsum)
        # channels with weight: divided by it; the rest (all zero) by 1 --
        # the same values as out[:, good] /= wsum[good], without the boolean
        # indexing's device-to-host round trip in every iteration
        out /= torch.where(wsum > 0, wsum, 1.0)[None, :, None]
        model_port = out[0]             # the next template stays in HBM
        niter -= 1
        count += 1
    aligned_port = out.cpu().numpy()
    total_weights = np.outer(wsum.cpu().numpy(), np.ones(nbin))
    if norm in ("mean", "max", "prof", "rms", "abs"):
        for ipol in range(npol):
            aligned_port[ipol] = normalize_portrait(aligned_port[ipol], norm,
                                                    weights=None)
    if rot_phase:
        aligned_port = rotate_data(aligned_port, rot_phase)
    if place is not None:
        prof = np.average(aligned_port[0], axis=0, weights=None)
        delta = prof.max() * gaussian_profile(len(prof), place, 0.0001)
        phase = fit_phase_shift(prof, delta, Ns=nbin).phase
        aligned_port = rotate_data(aligned_port, phase)
    try:
        arch = model_data.arch
    except (AttributeError, KeyError):
        arch = None
    if arch is not None and outfile is not None:    # ppalign.py:259-277
        arch.tscrunch()
        if pscrunch:
            arch.pscrunch()
        else:
            arch.convert_state("Stokes")
        arch.set_dispersion_measure(0.0)
        for subint in arch:
            for ipol in range(arch.get_npol()):
                for ichan in range(arch.get_nchan()):
                    prof = subint.get_Profile(ipol, ichan)
                    prof.get_amps()[:] = aligned_port[ipol, ichan]
                    if total_weights[ichan].sum() == 0.0:
                        subint.set_weight(ichan, 0.0)
                    else:
                        subint.set_weight(ichan, 1.0)
        arch.unload(outfile)
        if not quiet:
            print("\nUnloaded %s.\n" % outfile)
    return DataBunch(port=aligned_port, total_weights=total_weights,
                     nsub_fit=R.n)

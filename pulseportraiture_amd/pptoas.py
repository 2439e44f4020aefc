"""Drop-in mirror of PulsePortraiture's ``pptoas`` wideband-TOA driver.

``GetTOAs.get_TOAs`` keeps the reference signature and fills the same
attributes, but instead of fitting one sub-integration at a time it gathers
every usable sub-integration of an archive into ONE batched device call
(initial-phase FFTFIT + wideband fit + post-fit, ``ppf_fit_batch``) and then
does the unchanged per-sub-integration host bookkeeping (TOA epochs, Doppler
corrections, TOA flags, DeltaDM).  Archive I/O stays on PSRCHIVE via
``load_data`` (host side, out of the accelerated path).

Reference: /root/reference/pptoas.py (file:line cited per block).
"""
import contextlib
import ctypes
import gc
import os
import sys
import threading
import time
import warnings
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from . import _lib, engine
from . import dist as _dist
from . import pplib as _pplib
from .timeline import span
from .pplib import (DataBunch, file_is_type, guess_fit_freq, read_model,
                    scattering_alpha, write_TOAs, weighted_mean,
                    scattering_times, scattering_portrait_FT,
                    gen_gaussian_portrait, _raise_status, _box)
from . import pptoaslib as _pptl
from .pptoaslib import unpack_result, _status_message, _nu_zero_messages

max_nfile = 999                    # pptoas.py:33
rm_baseline = bool(_pplib.F0_fact)  # pptoas.py:36-39
# whole-array batch gathering and bookkeeping for archives whose fitted
# sub-ints share channels, frequencies and fit flags (bit-identical to the
# per-sub-int loops, which remain the general path; False forces those)
FAST_HOST = True
_SWITCH_MS = float(os.environ.get("PPF_SWITCH_INTERVAL_MS", "0") or 0)
# threads of the native pageable -> page-locked staging copy of in-memory
# archives (_Stager; 0: torch's copy_)
_STAGE_COPY_THREADS = max(0, min(64, int(os.environ.get(
    "PPF_STAGE_COPY_THREADS", "8"))))


def _is_fits(filename):
    try:
        return file_is_type(filename, "FITS")
    except (OSError, TypeError):
        return False


def load_data(filename, **kwargs):
    """Indirection so tests / users can supply archives without PSRCHIVE."""
    return _pplib.load_data(filename, **kwargs)


_PSRCHIVE = []


def _MJD(days):
    if not _PSRCHIVE:
        try:
            import psrchive as pr
            _PSRCHIVE.append(pr.MJD)
        except ImportError:
            _PSRCHIVE.append(_pplib.MJD)     # PSRCHIVE-free MJD arithmetic
    return _PSRCHIVE[0](days)


_MJD_ORIG = _MJD


def _MJD_is_plain():
    """True when TOA epochs are pplib.MJD: no PSRCHIVE bindings and _MJD
    not replaced (tests substitute their own epoch type)."""
    if _MJD is not _MJD_ORIG:
        return False
    _MJD(0.0)
    return bool(_PSRCHIVE) and _PSRCHIVE[0] is _pplib.MJD


def _rank_world():
    """(rank, world) when torch.distributed runs more than one rank."""
    if _dist.is_dist():
        import torch.distributed as tdist
        return tdist.get_rank(), tdist.get_world_size()
    return 0, 1


_WSTREAMS = {}
_WLOCK = threading.Lock()


def _worker_stream(dev):
    """The fit worker's own HIP stream (one per device)."""
    with _WLOCK:
        if dev.index not in _WSTREAMS:
            _WSTREAMS[dev.index] = torch.cuda.Stream(dev)
        return _WSTREAMS[dev.index]


class _Staged(object):
    def __init__(self, fut):
        self.fut = fut

    def wait(self):
        """The uploaded rows, ordered after the upload on the caller's
        current stream."""
        t, ev = self.fut.result()
        if ev is not None:
            cur = torch.cuda.current_stream(t.device)
            cur.wait_event(ev)
            t.record_stream(cur)
        return t

    def release(self):
        self.fut = None


class _OnDevice(object):
    """A staged batch that is already in HBM (the PSRFITS fast path's
    unpacked rows): the selected sub-ints, ordered after the unpack."""

    def __init__(self, rows, event, sel, nchan, nbin):
        self.rows, self.event, self.sel = rows, event, list(sel)
        self.nchan, self.nbin = nchan, nbin

    def wait(self):
        cur = torch.cuda.current_stream(self.rows.device)
        if self.event is not None:
            cur.wait_event(self.event)
        sel = self.sel
        if not sel:
            return torch.zeros((0, self.nchan, self.nbin), dtype=torch.float32,
                               device=self.rows.device)
        if sel == list(range(sel[0], sel[0] + len(sel))):
            t = self.rows[sel[0]:sel[0] + len(sel)]
        else:
            t = self.rows.index_select(0, torch.as_tensor(sel, device=self.rows.device))
        self.rows.record_stream(cur)
        return t

    def release(self):
        self.rows = None


class _Stager(object):
    """Host data plane of get_TOAs: an archive's rows are copied into one of
    two pinned host buffers (float32 when every amplitude survives the round
    trip, as PSRCHIVE stores them) and uploaded asynchronously on a copy
    stream, so the upload of archive i+1 overlaps the fit of archive i; a
    buffer is reused only after its previous upload has completed.  The
    copy into pinned memory and the upload run on a thread of their own, so
    the caller goes on to the next archive's host work at once."""

    def __init__(self):
        self.bufs, self.events, self.k = [None, None], [None, None], 0
        self.stream = None
        self.pool = ThreadPoolExecutor(max_workers=1)

    def stage(self, rows):
        """rows: an array [n, nchan, nbin] or a view of one (no copy is
        made before the one into pinned memory, which runs on torch's CPU
        thread pool: a single-threaded numpy copy of a 268 MB archive costs
        ~25 ms, more than its fit)."""
        dev = engine.device()
        return _Staged(self.pool.submit(self._stage, np.asarray(rows), dev))

    def _stage(self, rows, dev):
        src = torch.from_numpy(rows)
        if src.numel() and src.is_contiguous() and src.is_pinned():
            # the loader put the archive in page-locked memory
            # (engine.pinned_host_array): the copy engine reads it directly,
            # no host-side copy (the caller leaves it unchanged during
            # get_TOAs, as load_data's arrays are)
            with torch.cuda.device(dev):
                if self.stream is None:
                    self.stream = torch.cuda.Stream(dev)
                with torch.cuda.stream(self.stream):
                    t = src.to(dev, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
            return t, ev
        if src.dtype != torch.float32:
            src = src.to(torch.float64)
            s32 = src.to(torch.float32)
            if bool(torch.equal(s32.to(torch.float64), src)):
                src = s32
        if src.numel() == 0:
            return torch.zeros(tuple(src.shape), dtype=torch.float32,
                               device=dev), None
        k = self.k
        self.k ^= 1
        if self.events[k] is not None:
            self.events[k].synchronize()
        need = src.numel() * src.element_size()
        if self.bufs[k] is None or self.bufs[k].numel() < need:
            self.bufs[k] = torch.empty(need, dtype=torch.uint8,
                                       pin_memory=True)
        host = self.bufs[k][:need].view(src.dtype).view(src.shape)
        if _STAGE_COPY_THREADS > 0 and src.is_contiguous():
            # native parallel memcpy outside the interpreter lock
            # (ppf_host_copy; torch's copy_ reached 30-38 GB/s here, which
            # bounded float32 archives below the PCIe rate)
            rc = _lib.load().ppf_host_copy(
                ctypes.c_void_p(host.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                need, _STAGE_COPY_THREADS)
            if rc != 0:
                raise RuntimeError("ppf_host_copy failed (%d)" % rc)
        else:
            host.copy_(src)
        with torch.cuda.device(dev):
            if self.stream is None:
                self.stream = torch.cuda.Stream(dev)
            with torch.cuda.stream(self.stream):
                t = host.to(dev, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
        self.events[k] = ev
        return t, ev

    def close(self):
        self.pool.shutdown(wait=True)
        for ev in self.events:
            if ev is not None:
                ev.synchronize()
        self.bufs, self.events = [None, None], [None, None]


class MJDValue(object):
    """A picklable stand-in for a TOA epoch that cannot be pickled (a
    PSRCHIVE MJD is a SWIG object): the integer and fractional day
    write_TOAs prints (pplib.py:3612-3648), as the original object gave
    them."""

    def __init__(self, intday, fracday):
        self._i, self._f = int(intday), float(fracday)

    def intday(self):
        return self._i

    def fracday(self):
        return self._f

    def in_days(self):
        return self._i + self._f


def _picklable_toa(toa):
    import pickle
    try:
        pickle.dumps(toa.MJD)
    except Exception:
        toa.MJD = MJDValue(toa.MJD.intday(), toa.MJD.fracday())
    return toa


def _table_width(nchan):
    return _lib.RESULT_DOUBLES + 3 * nchan + 25


def _pack(res):
    """One row per sub-int: the result record, scales, scale_errs,
    channel_snrs and the 5x5 covariance (the table all-gathered across
    ranks)."""
    n = res["results"].shape[0]
    return torch.cat([res["results"], res["scales"], res["scale_errs"],
                      res["channel_snrs"], res["covariance"].reshape(n, 25)],
                     dim=1)


def _unflat(res, host):
    """engine.fit_batch's outputs as host arrays, cut from the download of
    their one device buffer (res["_flat"])."""
    out, o = {}, 0
    for k in ("results", "scales", "scale_errs", "channel_snrs",
              "covariance"):
        shape = tuple(res[k].shape)
        n = int(np.prod(shape))
        out[k] = host[o:o + n].reshape(shape)
        o += n
    return out


def _unpack(t, nchan):
    R = _lib.RESULT_DOUBLES
    return dict(results=t[:, :R], scales=t[:, R:R + nchan],
                scale_errs=t[:, R + nchan:R + 2 * nchan],
                channel_snrs=t[:, R + 2 * nchan:R + 3 * nchan],
                covariance=t[:, R + 3 * nchan:].reshape(-1, 5, 5))


class TOA(object):
    """pptoas.py:42-84."""

    def __init__(self, archive, frequency, MJD, TOA_error, telescope,
                 telescope_code, DM=None, DM_error=None, flags={}):
        self.archive = archive
        self.frequency = frequency
        self.MJD = MJD
        self.TOA_error = TOA_error
        self.telescope = telescope
        self.telescope_code = telescope_code
        self.DM = DM
        self.DM_error = DM_error
        self.flags = flags

    def write_TOA(self, inf_is_zero=True, outfile=None):
        write_TOAs(self, inf_is_zero=inf_is_zero, outfile=outfile,
                   append=True)


_ATTRS = ["obs", "doppler_fs", "nu0s", "nu_fits", "nu_refs", "ok_idatafiles",
          "ok_isubs", "epochs", "MJDs", "Ps", "phis", "phi_errs", "TOAs",
          "TOA_errs", "DM0s", "DMs", "DM_errs", "DeltaDM_means",
          "DeltaDM_errs", "GMs", "GM_errs", "taus", "tau_errs", "alphas",
          "alpha_errs", "scales", "scale_errs", "snrs", "channel_snrs",
          "profile_fluxes", "profile_flux_errs", "fluxes", "flux_errs",
          "flux_freqs", "red_chi2s", "channel_red_chi2s", "covariances",
          "nfevals", "rcs", "fit_durations", "order", "TOA_list",
          "zap_channels"]


class GetTOAs(object):
    """pptoas.py:87-159."""

    def __init__(self, datafiles, modelfile, quiet=False):
        if file_is_type(datafiles, "ASCII"):
            with open(datafiles) as fh:
                self.datafiles = [ln.rstrip("\n") for ln in fh.readlines()
                                  if ln.strip()]
        else:
            self.datafiles = [datafiles]
        if len(self.datafiles) > max_nfile:
            print("Too many archives.  See/change max_nfile(=%d) in pptoas.py."
                  % max_nfile)
            raise SystemExit
        self.is_FITS_model = file_is_type(modelfile, "FITS")
        self.modelfile = modelfile
        for a in _ATTRS:
            setattr(self, a, [])
        self.instrumental_response_dict = self.ird = \
            {"DM": 0.0, "wids": [], "irf_types": []}
        self.quiet = quiet

    # ------------------------------------------------------------------
    def _models(self, d, ok_isubs, fit_scat, quiet, host=True):
        """Model portrait per sub-integration (pptoas.py:385-419): the
        .gmodel is parsed once (read_model, pplib.py:2971-3057) and every
        distinct (frequency set, TAU [bin]) portrait of the archive is built
        in ONE ppf_gauss_portrait_batch launch (k_gauss_port)."""
        if self.is_FITS_model:
            raise NotImplementedError("FITS (archive) templates need PSRCHIVE")
        # within one get_TOAs call the template file is read once and an
        # archive whose portraits (frequency sets, TAU) equal an earlier
        # archive's reuses that archive's device portraits: the same
        # deterministic k_gauss_port output the reference rebuilds per
        # archive
        mc = self.__dict__.setdefault("_mcache", {})
        try:
            if "model" not in mc:
                mc["model"] = read_model(self.modelfile, quiet=True)
            (self.model_name, code, nu_ref, self.ngauss, gparams, _mff, alpha,
             _mfa) = mc["model"]
        except (UnboundLocalError, UnicodeDecodeError):
            # a make_spline_model template (pptoas.py:416-419): one device
            # portrait per distinct frequency set, unscattered
            return self._spline_models(d, ok_isubs, host)
        if fit_scat:
            (self.model_code, self.model_nu_ref, self.gparams,
             self.alpha) = code, nu_ref, gparams, alpha
        nbin = len(d.phases)
        cache, prms, freqs, index = {}, [], [], []
        g1 = gparams[1]
        for isub in ok_isubs:
            # TAU: 0 for the unscattered template of a scattering fit
            # (pptoas.py:408-417), else read_model's [s] -> [bin]
            t1 = 0.0 if fit_scat else (g1 * (nbin / d.Ps[isub])
                                       if g1 != 0.0 else g1)
            key = (d.freqs[isub].tobytes(), float(t1))
            if key not in cache:
                cache[key] = len(prms)
                p = np.copy(gparams)
                p[1] = t1
                prms.append(p)
                freqs.append(np.asarray(d.freqs[isub], dtype=float))
            index.append(cache[key])
        if not prms:
            return np.zeros((0, len(d.freqs[0]), nbin)), \
                np.zeros(0, dtype=np.int32)
        if nbin % 2 and any(p[1] != 0.0 for p in prms):
            # the reference's scattered model is the length-less irfft of
            # gen_gaussian_portrait (pplib.py:957): nbin - 1 bins at odd nbin,
            # then fitted against nbin-bin data (a transform of another
            # length); the batched fit takes one nbin for both, so refuse
            # rather than fit a zero-padded model
            raise NotImplementedError(
                "GetTOAs with a scattered Gaussian model (TAU != 0) at odd "
                "nbin = %d: the reference fits an nbin - 1 bin model there" %
                nbin)
        ck = (bool(fit_scat), nbin, tuple(cache))
        models = mc.get(ck)
        if models is None:
            models = engine.gauss_portraits(
                code, np.stack(prms), 0.0 if fit_scat else alpha,
                np.stack(freqs), nu_ref, nbin)
            if len(mc) > 8:
                mc.clear()
                mc["model"] = (self.model_name, code, nu_ref, self.ngauss,
                               gparams, _mff, alpha, _mfa)
            mc[ck] = models
        return (models.cpu().numpy() if host else models,
                np.array(index, dtype=np.int32))

    def _spline_models(self, d, ok_isubs, host=True):
        """read_spline_model(modelfile, freqs, nbin) per sub-integration
        (pptoas.py:416-419), the distinct frequency sets of the archive in
        ONE ppf_spline_portrait_batch launch."""
        from .pplib import read_spline_model
        (self.model_name, _src, _df, mean_prof, eigvec,
         tck) = read_spline_model(self.modelfile, quiet=True)
        nbin = len(d.phases)
        cache, freqs, index = {}, [], []
        for isub in ok_isubs:
            key = d.freqs[isub].tobytes()
            if key not in cache:
                cache[key] = len(freqs)
                freqs.append(np.asarray(d.freqs[isub], dtype=float))
            index.append(cache[key])
        if not freqs:
            return np.zeros((0, len(d.freqs[0]), nbin)), \
                np.zeros(0, dtype=np.int32)
        models = engine.spline_portraits(mean_prof, eigvec, tck,
                                         np.stack(freqs), nbin)
        return (models.cpu().numpy() if host else models,
                np.array(index, dtype=np.int32))

    def get_TOAs(self, datafile=None, tscrunch=False, nu_refs=None, DM0=None,
                 bary=True, fit_DM=True, fit_GM=False, fit_scat=False,
                 log10_tau=True, scat_guess=None, fix_alpha=False,
                 print_phase=False, print_flux=False, print_parangle=False,
                 add_instrumental_response=False, addtnl_toa_flags={},
                 method="trust-ncg", bounds=None, nu_fits=None,
                 show_plot=False, quiet=None):
        """pptoas.py:161-792, batched per archive on the GPU."""
        if quiet is None:
            quiet = self.quiet
        if show_plot:
            raise NotImplementedError("plotting is outside the accelerated "
                                      "path (SURVEY.md section 2, row 20)")
        if add_instrumental_response and (self.ird["DM"] or
                                          len(self.ird["wids"])):
            raise NotImplementedError("instrumental response (SURVEY.md row "
                                      "19) is not on the accelerated path")
        if method not in ("trust-ncg", "Newton-CG", "TNC"):
            print("Method '%s' is not implemented." % method)
            raise SystemExit
        already_warned = False
        warning_message = \
            "You are using an experimental functionality of pptoas!"
        self.nfit = 1 + int(fit_DM) + int(fit_GM) + 2 * int(fit_scat) - \
            int(fix_alpha)
        self.fit_phi = True
        self.fit_DM, self.fit_GM = fit_DM, fit_GM
        self.fit_tau = self.fit_alpha = fit_scat
        if fit_scat:
            self.fit_alpha = not fix_alpha
        self.fit_flags = [int(self.fit_phi), int(self.fit_DM),
                          int(self.fit_GM), int(self.fit_tau),
                          int(self.fit_alpha)]
        self.log10_tau = log10_tau
        if not fit_scat:
            self.log10_tau = log10_tau = False
        if self.fit_GM or fit_scat or self.fit_tau or self.fit_alpha:
            print(warning_message)
            already_warned = True
        self.scat_guess = scat_guess
        nu_ref_tuple, nu_fit_tuple = nu_refs, nu_fits
        self.DM0, self.bary = DM0, bary
        start = time.time()
        tot_duration = 0.0
        datafiles = self.datafiles if datafile is None else [datafile]
        self.tscrunch = tscrunch
        self.add_instrumental_response = add_instrumental_response
        self._ff = [None]   # fit_flags carried across sub-ints (pptoas.py:519-529)
        self._mcache = {}   # template portraits of this call (_models)
        self._fit_ws = {}   # the fit worker's workspace (_fit_share)
        # With several ranks and at least as many archives as ranks, each
        # rank loads and fits only its own contiguous block of archives
        # (pptoas.py:258) and the per-archive results are
        # gathered at the end; a single archive (or fewer archives than
        # ranks) is sharded by sub-int instead (_prep_archive).  So is a
        # fit_DM + fit_GM run: its fit_flags list carries over from one
        # archive to the next (the 2-channel rule, pptoas.py:523-525), which
        # only a rank that has seen every earlier archive can reproduce.
        rank, world = _rank_world()
        # (nor method='TNC' without bounds: its default tau bound comes from
        # the nbin of the first sub-int fitted in serial order,
        # pptoas.py:503-513, which a rank starting at a later archive cannot
        # see)
        by_archive = world > 1 and len(datafiles) >= world and \
            not (self.fit_DM and self.fit_GM) and \
            not (method == "TNC" and bounds is None)
        mine = range(len(datafiles))
        if by_archive:
            a0, na = _dist.shard(len(datafiles), rank, world)
            mine = range(a0, a0 + na)
            marks = {a: len(getattr(self, a)) for a in _ATTRS}
        ctx = dict(quiet=quiet, tscrunch=tscrunch, fit_scat=fit_scat,
                   method=method, bounds=[bounds], by_archive=by_archive,
                   nu_fit_tuple=nu_fit_tuple, nu_ref_tuple=nu_ref_tuple,
                   bary=bary, print_phase=print_phase, print_flux=print_flux,
                   print_parangle=print_parangle,
                   addtnl_toa_flags=addtnl_toa_flags)
        # Two-stage pipeline (the host data plane): while the device fits
        # archive i (a worker thread on its own HIP stream; ppf_fit_batch
        # releases the GIL), this thread loads archive i+1, builds its batch
        # and starts its upload from pinned memory on a copy stream; then it
        # does archive i's bookkeeping.
        stager = _Stager()
        pool = ThreadPoolExecutor(max_workers=1)
        # load_data of archive i+1 runs on a loader thread while archive i
        # is prepared (a PSRFITS archive's file read, upload and device
        # unpack: psrfits.load_data, whose reads and copies release the
        # GIL); the reference's first load_data call, made ahead of time,
        # with the same arguments.  PPF_LOAD_DEPTH loads more archives at
        # once on as many threads: measured slower (16-bit PSRFITS, 32
        # archives: depth 1 6.1-6.2k, 2 5.1-5.6k, 3 4.7-5.3k TOAs/s in one
        # call; the file reads and pinned copies share the host's memory
        # bandwidth).  PPF_LOAD_AHEAD archives are queued ahead on those
        # threads (a PSRFITS load parses the file and hands the read to the
        # reader threads, so the one loader thread keeps going): 3 ahead
        # with psrfits' 4 pinned slots 17.5-18.1k vs 2 ahead / 3 slots
        # 15.6-17.1k TOAs/s (A/B in one call, tools/g21.sh)
        depth = max(1, int(os.environ.get("PPF_LOAD_DEPTH", "1")))
        ahead_n = max(depth, int(os.environ.get("PPF_LOAD_AHEAD", "3")))
        loader = ThreadPoolExecutor(max_workers=depth)
        mine = list(mine)
        loads = {}

        # the loader thread works on this rank's device: the HIP current
        # device is per host thread, and a new thread starts on GPU 0
        ldev = engine.device() if torch.cuda.is_available() else None

        def _load(f):
            # defer + lazy: a PSRFITS file is parsed and its DATA read
            # started here; the read thread queues its upload and device
            # work when the read completes (psrfits._Pending), while this
            # thread goes on to parse the next file; _prep_archive's finish()
            # waits for them
            with (torch.cuda.device(ldev) if ldev is not None else
                  contextlib.nullcontext()):
                return load_data(f, dedisperse=False, dededisperse=False,
                                 tscrunch=tscrunch, pscrunch=True,
                                 fscrunch=False, rm_baseline=rm_baseline,
                                 flux_prof=False, refresh_arch=False,
                                 return_arch=False, quiet=quiet,
                                 **({"defer": True, "lazy": True}
                                    if _is_fits(f) else {}))
        pending = None
        err = None
        # the cyclic garbage collector is paused for the loop (restored
        # after): get_TOAs allocates a few objects per TOA that form no
        # cycles, and a full collection over a large TOA list is a
        # millisecond pause in whichever stage it lands
        gc_on = gc.isenabled()
        gc.disable()
        # the interpreter's thread switch interval for the loop (env
        # PPF_SWITCH_INTERVAL_MS; unset: left as it is)
        sw0 = sys.getswitchinterval()
        if _SWITCH_MS:
            sys.setswitchinterval(_SWITCH_MS * 1e-3)
        try:
            for pos, iarch in enumerate(mine):
                for ahead in range(ahead_n + 1):
                    if pos + ahead < len(mine) and mine[pos + ahead] not in loads:
                        nxt = mine[pos + ahead]
                        loads[nxt] = loader.submit(_load, datafiles[nxt])
                with span("prep"):
                    job = self._prep_archive(iarch, datafiles[iarch], ctx,
                                             stager, loads.pop(iarch))
                if job is None:
                    continue
                fut = pool.submit(self._fit_archive, job, ctx)
                if pending is not None:
                    with span("main.wait_fit"):
                        r = pending[1].result()
                    with span("book"):
                        self._book_archive(pending[0], r, ctx, start)
                pending = (job, fut)
            if pending is not None:
                with span("main.wait_fit"):
                    r = pending[1].result()
                with span("book"):
                    self._book_archive(pending[0], r, ctx, start)
        except Exception as exc:            # every rank raises, below
            if not by_archive:
                raise
            err = exc
        finally:
            if gc_on:
                gc.enable()
            sys.setswitchinterval(sw0)
            pool.shutdown(wait=True)
            for fu in loads.values():
                fu.cancel()
            loader.shutdown(wait=True)
            stager.close()
        if by_archive:
            # a failed rank must not leave the others in the gather
            _dist.raise_if_any_failed(err, ldev)
            self._gather_archives(marks)

    def _gather_archives(self, marks):
        """Archive-sharded get_TOAs: every rank's per-archive results (one
        entry per archive in each per-archive attribute, the archive's TOAs)
        are all-gathered as objects and re-assembled in archive order, so
        every rank ends with the attributes and TOA list of a serial run."""
        import torch.distributed as tdist
        per = [a for a in _ATTRS if a not in ("ok_idatafiles", "TOA_list",
                                              "channel_red_chi2s",
                                              "zap_channels")]
        mine = self.ok_idatafiles[marks["ok_idatafiles"]:]
        recs = []
        ntoa = [len(np.asarray(v)) for v in self.ok_isubs[marks["ok_isubs"]:]]
        toas = self.TOA_list[marks["TOA_list"]:]
        pos = 0
        for j, iarch in enumerate(mine):
            rec = {a: getattr(self, a)[marks[a] + j] for a in per}
            rec["_toas"] = [_picklable_toa(t) for t in toas[pos:pos + ntoa[j]]]
            rec["_iarch"] = iarch
            pos += ntoa[j]
            recs.append(rec)
        allrecs = [None] * tdist.get_world_size()
        tdist.all_gather_object(allrecs, recs)
        merged = sorted((r for rr in allrecs for r in rr),
                        key=lambda r: r["_iarch"])
        for a in _ATTRS:
            del getattr(self, a)[marks[a]:]
        for r in merged:
            self.ok_idatafiles.append(r["_iarch"])
            for a in per:
                getattr(self, a).append(r[a])
            self.TOA_list.extend(r["_toas"])

    # ------------------------------------------------------------------
    def _prep_archive(self, iarch, datafile, ctx, stager, loaded=None):
        """Load one archive and build its batch (pptoas.py:258-529); None if
        the archive is skipped.  loaded: the future of load_data(datafile)
        already started ahead (get_TOAs' loader thread)."""
        quiet, tscrunch, fit_scat = ctx["quiet"], ctx["tscrunch"], \
            ctx["fit_scat"]
        nu_fit_tuple, nu_ref_tuple, bary = ctx["nu_fit_tuple"], \
            ctx["nu_ref_tuple"], ctx["bary"]
        fit_duration = 0.0
        try:
            if loaded is not None:
                with span("prep.wait_load"):
                    data = loaded.result()
                    fin = getattr(data, "finish", None)
                    if fin is not None and not isinstance(data, dict):
                        data = fin()
            else:
                data = load_data(datafile, dedisperse=False,
                                 dededisperse=False, tscrunch=tscrunch,
                                 pscrunch=True, fscrunch=False,
                                 rm_baseline=rm_baseline, flux_prof=False,
                                 refresh_arch=False, return_arch=False,
                                 quiet=quiet)
            if data.dmc:
                if not quiet:
                    print("%s is dedispersed (dmc = 1).  Reloading it." %
                          datafile)
                data = load_data(datafile, dedisperse=False,
                                 dededisperse=True, tscrunch=tscrunch,
                                 pscrunch=True, fscrunch=False,
                                 rm_baseline=rm_baseline,
                                 flux_prof=False, refresh_arch=False,
                                 return_arch=False, quiet=quiet)
            if np.isnan(data.prof_SNR) or (data.prof_SNR == 0.0):
                print("Profile has a nan or zero  snr, must skip")
                return None
            nnan = len(data.SNRs[np.isnan(data.SNRs)])
            if nnan > 10:
                print("More than 10 frequency channels with nan SNR. "
                      "Skipping it")
                return None
            if nnan > 0:
                print("This file has %s frequency channels with a nan SNR"
                      % nnan)
                print(datafile)
                for isub in data.ok_isubs:
                    for ipol in range(data.npol):
                        oc = np.array(data.ok_ichans[isub])
                        data.ok_ichans[isub] = oc[~np.isnan(
                            data.SNRs[isub, ipol][oc])]
            if not len(data.ok_isubs):
                if not quiet:
                    print("No subints to fit for %s.  Skipping it." %
                          datafile)
                return None
            self.ok_idatafiles.append(iarch)
        except RuntimeError:
            if not quiet:
                print("Cannot load_data(%s).  Skipping it." % datafile)
            return None
        d = data
        nsub, nchan, nbin = d.nsub, d.nchan, d.nbin
        if bary and not d.get("doppler_known", True) and \
                not ctx.get("bary_warned"):
            # psrfits.load_data has no ephemeris: its Doppler factors are 1
            # (warned once per get_TOAs call, naming the first such archive)
            ctx["bary_warned"] = True
            warnings.warn("%s: Doppler factors unknown on the PSRFITS fast "
                          "path (no PSRCHIVE ephemeris); DM, GM and nu_ref_tau "
                          "stay topocentric (bary=True has no effect)" %
                          datafile, RuntimeWarning)
        if d.source is None:
            d.source = "noname"
        obs = DataBunch(telescope=d.telescope, backend=d.backend,
                        frontend=d.frontend)
        nu_fits_a = list(np.zeros([nsub, 3], dtype=np.float64))
        nu_refs_a = list(np.zeros([nsub, 3], dtype=np.float64))
        MJDs = np.array([d.epochs[isub].in_days() for isub in range(nsub)],
                        dtype=np.double)
        DM_stored = d.DM
        DM0 = DM_stored if self.DM0 is None else self.DM0
        if not quiet:
            print("\nEach of the %d TOAs is approximately %.2f s" % (
                len(d.ok_isubs), d.integration_length / nsub))
        ok_isubs = list(d.ok_isubs)
        nok = len(ok_isubs)
        # the portraits stay in HBM: the fit worker orders itself after
        # their generation on this thread's stream (models_ev)
        _sp = span("prep.models")
        _sp.__enter__()
        models, model_index = self._models(d, ok_isubs, fit_scat, quiet,
                                           host=False)
        models_ev = None
        if isinstance(models, torch.Tensor) and models.is_cuda:
            models_ev = torch.cuda.Event()
            models_ev.record(torch.cuda.current_stream(models.device))
        _sp.__exit__(None, None, None)
        _sp = span("prep.batch")
        _sp.__enter__()
        fast = self._gather_uniform(d, ok_isubs, ctx, nu_fits_a, nu_refs_a,
                                    DM_stored) if FAST_HOST else None
        if fast is not None:
            mask, init, flags_b, nu_fit_b, nu_out_b, guess_tau = fast
        else:
            mask, init, flags_b, nu_fit_b, nu_out_b, guess_tau = \
                self._gather_rows(d, ok_isubs, ctx, nu_fits_a, nu_refs_a,
                                  DM_stored)
        _sp.__exit__(None, None, None)
        rank, world = (0, 1) if ctx["by_archive"] else _rank_world()
        first, count = _dist.shard(nok, rank, world)
        sel = ok_isubs[first:first + count]
        dev_rows = getattr(d.subints, "device_rows", None)
        if dev_rows is not None:
            # PSRFITS fast path: the rows were unpacked on the device by
            # load_data (psrfits.load_data); no host copy, no second upload
            staged = _OnDevice(dev_rows, d.subints.event, sel, nchan, nbin)
        else:
            staged = None
        if staged is not None:
            rows = None
        elif count and sel == list(range(sel[0], sel[0] + count)):
            # contiguous sub-ints (the usual case): a view, no gather copy
            rows = np.asarray(d.subints)[sel[0]:sel[0] + count, 0]
        elif count:
            rows = np.asarray(d.subints)[sel, 0]
        else:
            rows = np.zeros((0, nchan, nbin))
        return dict(iarch=iarch, datafile=datafile, d=d, nsub=nsub,
                    dev=engine.device(),
                    nchan=nchan, nbin=nbin, obs=obs, nu_fits_a=nu_fits_a,
                    nu_refs_a=nu_refs_a, MJDs=MJDs, DM_stored=DM_stored,
                    DM0=DM0, ok_isubs=ok_isubs, nok=nok, models=models,
                    models_ev=models_ev,
                    model_index=model_index, mask=mask, init=init,
                    flags_b=flags_b, nu_fit_b=nu_fit_b, nu_out_b=nu_out_b,
                    guess_tau=guess_tau, first=first, count=count,
                    bounds=ctx["bounds"][0],
                    world=world,
                    staged=staged if staged is not None else stager.stage(rows),
                    fit_duration=fit_duration)

    def _tau_guess(self, P, nu_fit_tau, nbin):
        """pptoas.py:461-480: the initial scattering time (and index) of a
        sub-int; returns (tau_guess linear, init tau, alpha_guess)."""
        if self.scat_guess is not None:
            tg_s, tg_ref, alpha_guess = self.scat_guess
            tau_guess = (tg_s / P) * (nu_fit_tau / tg_ref) ** alpha_guess
        else:
            alpha_guess = self.alpha if hasattr(self, "alpha") \
                else scattering_alpha
            tau_guess = (self.gparams[1] / P) * (
                nu_fit_tau / self.model_nu_ref) ** alpha_guess \
                if hasattr(self, "gparams") else 0.0
        lin = tau_guess
        if self.log10_tau:
            if tau_guess == 0.0:
                tau_guess = nbin ** -1
            tau_guess = np.log10(tau_guess)
        return lin, tau_guess, alpha_guess

    def _set_tnc_bounds(self, ctx, nbin):
        if ctx["bounds"][0] is None and ctx["method"] == "TNC":
            # pptoas.py:503-513: set once, at the first sub-int fitted
            ctx["bounds"][0] = [
                (None, None), (None, None), (None, None),
                (0.0, None) if not self.log10_tau else
                (np.log10((10 * nbin) ** -1), None), (-10.0, 10.0)]

    def _gather_uniform(self, d, ok_isubs, ctx, nu_fits_a, nu_refs_a,
                        DM_stored):
        """_gather_rows for the usual archive, in whole-array operations:
        every fitted sub-int has the same usable channels (at least 3, so
        the 1/2-channel flag rules of pptoas.py:519-529 do not apply) and the
        same channel frequencies.  The values are bit-identical to the
        per-sub-int loop (guess_fit_freq's sums are the same pairwise row
        sums; tests/test_host_logic.py checks it).  None when the archive is
        not of that kind."""
        nok = len(ok_isubs)
        if not nok:
            return None
        oks = [d.ok_ichans[isub] for isub in ok_isubs]
        ok = np.asarray(oks[0], dtype=int)
        if len(ok) < 3 or not all(o is oks[0] or np.array_equal(o, ok)
                                  for o in oks[1:]):
            return None
        rows = np.asarray(ok_isubs)
        F = np.asarray(d.freqs)[rows]
        if not (F == F[0]).all():
            return None
        nchan, nbin = d.nchan, d.nbin
        nu_fit_tuple, nu_ref_tuple = ctx["nu_fit_tuple"], ctx["nu_ref_tuple"]
        mask = np.zeros((nok, nchan), dtype=np.uint8)
        mask[:, ok] = 1
        if nu_fit_tuple is None:
            # guess_fit_freq (pplib.py:2715-2729) of every row at once
            freqsx = F[0, ok]
            nu0 = (freqsx.min() + freqsx.max()) * 0.5
            w = np.asarray(d.SNRs)[rows, 0][:, ok] * freqsx ** -2
            nu_fit = nu0 + np.sum((freqsx - nu0) * w, axis=1) / \
                np.sum(w, axis=1)
            nf = [(v, v, v) for v in nu_fit]
        else:
            nf = [(nu_fit_tuple[0], nu_fit_tuple[0], nu_fit_tuple[-1])] * nok
        nu_fit_b = np.array(nf, dtype=float).reshape(nok, 3)
        nu_out_b = np.full((nok, 3), np.nan)
        bary = ctx["bary"]
        for j, isub in enumerate(ok_isubs):
            nu_fits_a[isub] = list(nf[j])
            if nu_ref_tuple is None:
                nu_refs_a[isub] = [None, None, None]
            else:
                nu_ref_tau = nu_ref_tuple[-1]
                if bary and nu_ref_tau:
                    nu_ref_tau /= d.doppler_factors[isub]
                nu_refs_a[isub] = [nu_ref_tuple[0], nu_ref_tuple[0],
                                   nu_ref_tau]
                nu_out_b[j] = [np.nan if v is None else v for v in
                               nu_refs_a[isub]]
        init = np.zeros((nok, 5))
        init[:, 1] = DM_stored
        guess_tau = np.zeros(nok)
        if ctx["fit_scat"]:
            for j, isub in enumerate(ok_isubs):
                guess_tau[j], init[j, 3], init[j, 4] = self._tau_guess(
                    d.Ps[isub], nf[j][2], nbin)
        self._set_tnc_bounds(ctx, nbin)
        self._ff[0] = list(np.copy(self.fit_flags))
        flags_b = np.zeros((nok, 5), dtype=np.int32)
        flags_b[:] = self._ff[0]
        return mask, init, flags_b, nu_fit_b, nu_out_b, guess_tau

    def _gather_rows(self, d, ok_isubs, ctx, nu_fits_a, nu_refs_a, DM_stored):
        """The batch's per-sub-int inputs (pptoas.py:384-529), one sub-int
        at a time."""
        quiet, fit_scat = ctx["quiet"], ctx["fit_scat"]
        nu_fit_tuple, nu_ref_tuple, bary = ctx["nu_fit_tuple"], \
            ctx["nu_ref_tuple"], ctx["bary"]
        nok, nchan, nbin = len(ok_isubs), d.nchan, d.nbin
        mask = np.zeros((nok, nchan), dtype=np.uint8)
        init = np.zeros((nok, 5))
        flags_b = np.zeros((nok, 5), dtype=np.int32)
        nu_fit_b = np.zeros((nok, 3))
        nu_out_b = np.full((nok, 3), np.nan)
        guess_tau = np.zeros(nok)
        for j, isub in enumerate(ok_isubs):
            ok = np.asarray(d.ok_ichans[isub], dtype=int)
            mask[j, ok] = 1
            freqsx = d.freqs[isub, ok]
            SNRsx = d.SNRs[isub, 0, ok]
            P = d.Ps[isub]
            if nu_fit_tuple is None:
                nu_fit = guess_fit_freq(freqsx, SNRsx)
                nu_fit_DM = nu_fit_GM = nu_fit_tau = nu_fit
            else:
                nu_fit_DM = nu_fit_GM = nu_fit_tuple[0]
                nu_fit_tau = nu_fit_tuple[-1]
            nu_fits_a[isub] = [nu_fit_DM, nu_fit_GM, nu_fit_tau]
            nu_fit_b[j] = nu_fits_a[isub]
            if nu_ref_tuple is None:
                nu_ref_DM = nu_ref_GM = nu_ref_tau = None
            else:
                nu_ref_DM = nu_ref_GM = nu_ref_tuple[0]
                nu_ref_tau = nu_ref_tuple[-1]
                if bary and nu_ref_tau:
                    nu_ref_tau /= d.doppler_factors[isub]
            nu_refs_a[isub] = [nu_ref_DM, nu_ref_GM, nu_ref_tau]
            nu_out_b[j] = [np.nan if v is None else v for v in
                           nu_refs_a[isub]]
            tau_guess = alpha_guess = 0.0
            if fit_scat:
                guess_tau[j], tau_guess, alpha_guess = self._tau_guess(
                    P, nu_fit_tau, nbin)
            init[j] = [0.0, DM_stored, 0.0, tau_guess, alpha_guess]
            self._set_tnc_bounds(ctx, nbin)
            # the reference's fit_flags is one list that lives across
            # sub-ints and archives: the 2-channel rule edits whatever the
            # previous sub-int left in it (pptoas.py:519-529, SURVEY.md
            # appendix B)
            if len(freqsx) == 1:
                self._ff[0] = [1, 0, 0, 0, 0]
                if not quiet:
                    print("TOA #%d only has 1 frequency channel...fitting "
                          "for phase only..." % (j + 1))
            elif len(freqsx) == 2 and self.fit_DM and self.fit_GM:
                if self._ff[0] is None:
                    raise UnboundLocalError(
                        "local variable 'fit_flags' referenced before "
                        "assignment (pptoas.py:525)")
                self._ff[0][2] = 0
                if not quiet:
                    print("TOA #%d only has 2 frequency channels...fitting "
                          "for phase and DM only..." % (j + 1))
            else:
                self._ff[0] = list(np.copy(self.fit_flags))
            flags_b[j] = self._ff[0]
        return mask, init, flags_b, nu_fit_b, nu_out_b, guess_tau

    def _fit_archive(self, job, ctx):
        """Device stage (worker thread): this rank's share of the archive's
        sub-ints in ONE ppf_fit_batch (guess + fit + post-fit), the result
        tables all-gathered over ranks; returns numpy tables."""
        d, nok, first, count = job["d"], job["nok"], job["first"], \
            job["count"]
        sl = slice(first, first + count)
        isubs = job["ok_isubs"][sl]
        nchan = job["nchan"]
        t_fit = time.time()
        dev = job["dev"]
        nccl = _dist.backend() == "nccl"
        with torch.cuda.device(dev), torch.cuda.stream(_worker_stream(dev)):
            with span("fit.wait_staged"):
                data_t = job["staged"].wait()
            _sp = span("fit.batch")
            _sp.__enter__()
            if job.get("models_ev") is not None:
                cur = torch.cuda.current_stream(dev)
                cur.wait_event(job["models_ev"])
                job["models"].record_stream(cur)
            err = None
            try:
                table = self._fit_share(job, ctx, data_t, isubs, sl, dev)
            except Exception as exc:        # every rank raises, below
                if job["world"] == 1:
                    raise
                err = exc
            if job["world"] > 1:
                # a failed rank must not leave the others in the all-gather
                _dist.raise_if_any_failed(err, dev if nccl else None)
                table = _pack(table) if isinstance(table, dict) else table
                table = _dist.allgather_rows(table if nccl else table.cpu(),
                                             nok, job["world"])
            with span("fit.d2h"):
                if isinstance(table, dict):
                    # one rank: the outputs' single buffer in one copy
                    r = _unflat(table, table["_flat"].cpu().numpy())
                else:
                    r = _unpack(table.cpu().numpy(), nchan)
            _sp.__exit__(None, None, None)
        job["staged"].release()
        r["batch_duration"] = time.time() - t_fit
        return r

    def _fit_share(self, job, ctx, data_t, isubs, sl, dev):
        """One ppf_fit_batch over this rank's sub-ints -> packed table."""
        d, count, nchan = job["d"], job["count"], job["nchan"]
        if not count:
            return torch.zeros((0, _table_width(nchan)), dtype=torch.float64,
                               device=dev)
        _sp = span("fit.call")
        _sp.__enter__()
        ws = self.__dict__.setdefault("_fit_ws", {})
        res = engine.fit_batch(
            data_t, job["models"], d.freqs[isubs], d.Ps[isubs],
            job["init"][sl], job["flags_b"][sl], nu_fits=job["nu_fit_b"][sl],
            nu_outs=job["nu_out_b"][sl],
            errs=np.asarray(d.noise_stds)[isubs, 0],
            chan_mask=job["mask"][sl], model_index=job["model_index"][sl],
            log10_tau=self.log10_tau, option=0, is_toa=True, guess=True,
            guess_weights=np.asarray(d.weights)[isubs],
            guess_DM=np.full(count, job["DM_stored"]), guess_Ns=100,
            guess_tau=job["guess_tau"][sl] if ctx["fit_scat"] else None,
            bounds=_box(job["bounds"], 5) if ctx["method"] == "TNC" else None,
            dev=dev, workspace=ws.get(dev), max_workspace=ws.get("max"))
        # the workspace is reused by the next archive's call on this (the
        # worker's) stream; the budget is the free HBM at the first call
        ws[dev] = res.get("workspace")
        if "max" not in ws and torch.cuda.is_available():
            ws["max"] = torch.cuda.mem_get_info(dev)[0] // 2
        _sp.__exit__(None, None, None)
        return res if "_flat" in res else _pack(res)

    def _book_uniform(self, job, r, ctx, fit_duration, out):
        """_book_archive's per-sub-int loop for an archive fitted with one
        set of fit flags (and no flux): the result columns are scattered in
        whole-array operations, only the TOA objects are built per sub-int.
        Bit-identical to the loop (tests/test_host_logic.py); returns the
        summed fit duration."""
        d, datafile = job["d"], job["datafile"]
        ok_isubs, nok = job["ok_isubs"], job["nok"]
        nu_refs_a, mask = job["nu_refs_a"], job["mask"]
        nchan, nbin = job["nchan"], job["nbin"]
        ff = [int(v) for v in job["flags_b"][0]]
        I = _lib.RESULT_INDEX
        Rt = r["results"]
        st = Rt[:, I["status"]].astype(np.int64)
        # the messages and failures of the loop, in its order
        nz_text = _pptl._nu_zero_text(ff)
        for j, isub in enumerate(ok_isubs):
            if nz_text is not None and not all(nu_refs_a[isub]):
                print(nz_text)
            s = int(st[j])
            _raise_status(s)
            if (s & 0xff) not in (0, 1, 2, 4):
                _status_message(s & 0xff, datafile + "_%d" % isub)
        dur = r["batch_duration"] / nok
        for _ in range(nok):
            fit_duration += dur
        rows = np.asarray(ok_isubs)
        okb = mask.astype(bool)
        params, perrs = Rt[:, I["params"]], Rt[:, I["param_errs"]]
        nuo = Rt[:, I["nu_out"]]
        DMv, GMv = params[:, 1].copy(), params[:, 2].copy()
        if self.bary:
            dfs = np.asarray(d.doppler_factors)[rows]
            if ff[1]:
                DMv *= dfs
            if ff[2]:
                GMv *= np.array([df ** 3 for df in dfs])
        out["phis"][rows], out["phi_errs"][rows] = params[:, 0], perrs[:, 0]
        out["DMs"][rows], out["DM_errs"][rows] = DMv, perrs[:, 1]
        out["GMs"][rows], out["GM_errs"][rows] = GMv, perrs[:, 2]
        out["taus"][rows], out["tau_errs"][rows] = params[:, 3], perrs[:, 3]
        out["alphas"][rows], out["alpha_errs"][rows] = params[:, 4], \
            perrs[:, 4]
        out["nfevals"][rows] = Rt[:, I["nfeval"]].astype(int)
        out["rcs"][rows] = st & 0xff
        # every channel usable (the common archive): plain copies; a
        # contiguous run of sub-ints: slices instead of gathers
        allok = bool(okb.all())
        rs = slice(int(rows[0]), int(rows[-1]) + 1) \
            if int(rows[-1]) - int(rows[0]) + 1 == nok else rows
        for key in ("scales", "scale_errs", "channel_snrs"):
            out[key][rs] = r[key] if allok else np.where(okb, r[key], 0.0)
        out["snrs"][rows] = Rt[:, I["snr"]]
        out["red_chi2s"][rows] = Rt[:, I["red_chi2"]]
        nfit = self.nfit
        out["covariances"][rs] = r["covariance"][:, :nfit, :nfit]
        F = np.asarray(d.freqs)[rs]
        if allok:
            nchx = np.full(nok, nchan)
            fmax, fmin = F.max(axis=1), F.min(axis=1)
        else:
            nchx = okb.sum(axis=1)
            fmax = np.where(okb, F, -np.inf).max(axis=1)
            fmin = np.where(okb, F, np.inf).min(axis=1)
        snr_c, gof_c = Rt[:, I["snr"]], Rt[:, I["red_chi2"]]
        cov01 = ctx["nu_ref_tuple"] is not None and all(ff[:2])
        common = [("be", d.backend), ("fe", d.frontend),
                  ("f", d.frontend + "_" + d.backend), ("nbin", nbin),
                  ("nch", nchan)]
        chbw = abs(d.bw) / nchan
        TOAs, TOA_errs = out["TOAs"], out["TOA_errs"]
        print_flux = ctx["print_flux"]
        if print_flux:
            mmean, model_index = out["mmean"], job["model_index"]
            pf, pfe = out["profile_fluxes"], out["profile_flux_errs"]
            scl, scle = r["scales"], r["scale_errs"]
            for j, isub in enumerate(ok_isubs):
                ok = okb[j]
                smm = mmean[model_index[j]][ok]
                pf[isub, ok] = smm * scl[j][ok]
                pfe[isub, ok] = abs(smm) * scle[j][ok]
                out["fluxes"][isub], out["flux_errs"][isub] = weighted_mean(
                    pf[isub, ok], pfe[isub, ok])
                out["flux_freqs"][isub], _ = weighted_mean(F[j][ok],
                                                           pfe[isub, ok])
        # the TOA epochs, in whole arrays: epoch + MJD((phi P + backend
        # delay) / 86400), the same additions and floors pplib.MJD makes
        # one TOA at a time (pptoas.py:578-580)
        Ps_r = np.asarray(d.Ps)[rows]
        dd = (params[:, 0] * Ps_r + d.backend_delay) / (3600 * 24.)
        toa_err = perrs[:, 0] * Ps_r * 1e6
        eps = [d.epochs[i] for i in ok_isubs]
        if _MJD_is_plain() and all(type(e) is _pplib.MJD for e in eps):
            mi = np.floor(dd)
            F = np.array([e._f for e in eps]) + (dd - mi)
            K = np.floor(F)
            I = np.array([e._i for e in eps], dtype=np.int64) + \
                mi.astype(np.int64) + K.astype(np.int64)
            toas = [_pplib.MJD._make(i, f) for i, f in zip(I.tolist(),
                                                          (F - K).tolist())]
        else:
            toas = [e + _MJD(x) for e, x in zip(eps, dd)]
        # the flag columns (one value per TOA, in the reference's key order)
        keys, cols = [], []

        def col(k, v):
            keys.append(k)
            cols.append(v)
        Pl, errl = list(Ps_r), list(toa_err)
        if self.bary:
            dfl = list(np.asarray(d.doppler_factors)[rows])
        else:
            dfl = [1.0] * nok
        if ff[2]:
            col("gm", list(GMv))
            col("gm_err", list(perrs[:, 2]))
        if ff[3]:
            taus_l, terr_l = list(params[:, 3]), list(perrs[:, 3])
            if self.log10_tau:
                col("scat_time", [10 ** t * P / df * 1e6 for t, P, df in
                                  zip(taus_l, Pl, dfl)])
                col("log10_scat_time", [t + np.log10(P / df) for t, P, df in
                                        zip(taus_l, Pl, dfl)])
                col("log10_scat_time_err", terr_l)
            else:
                col("scat_time", [t * P / df * 1e6 for t, P, df in
                                  zip(taus_l, Pl, dfl)])
                col("scat_time_err", [e * P / df * 1e6 for e, P, df in
                                      zip(terr_l, Pl, dfl)])
            col("scat_ref_freq", [v * df for v, df in zip(list(nuo[:, 2]),
                                                          dfl)])
            col("scat_ind", list(params[:, 4]))
        if ff[4]:
            col("scat_ind_err", list(perrs[:, 4]))
        for k, v in common:
            col(k, [v] * nok)
        col("nchx", nchx.tolist())
        col("bw", list(fmax - fmin))
        col("chbw", [chbw] * nok)
        col("subint", list(ok_isubs))
        col("tobs", [d.subtimes[i] for i in ok_isubs])
        col("fratio", list(fmax / fmin))
        col("tmplt", [self.modelfile] * nok)
        col("snr", list(snr_c))
        if cov01:
            col("phi_DM_cov", list(r["covariance"][:, 0, 1]))
        col("gof", list(gof_c))
        if ctx["print_phase"]:
            col("phs", list(params[:, 0]))
            col("phs_err", list(perrs[:, 0]))
        if print_flux:
            col("flux", [out["fluxes"][i] for i in ok_isubs])
            col("flux_err", [out["flux_errs"][i] for i in ok_isubs])
            col("flux_ref_freq", [out["flux_freqs"][i] for i in ok_isubs])
        if ctx["print_parangle"]:
            col("par_angle", [d.parallactic_angles[i] for i in ok_isubs])
        for k, v in ctx["addtnl_toa_flags"].items():
            col(k, [v] * nok)
        nul = [list(v) for v in nuo]
        DMl = list(DMv) if ff[1] else [None] * nok
        DMel = list(perrs[:, 1]) if ff[1] else [None] * nok
        tel, code = d.telescope, d.telescope_code
        for j, (isub, vals) in enumerate(zip(ok_isubs, zip(*cols))):
            nu_refs_a[isub] = nul[j]
            TOAs[isub], TOA_errs[isub] = toas[j], errl[j]
            self.TOA_list.append(TOA(datafile, nul[j][0], toas[j], errl[j],
                                     tel, code, DMl[j], DMel[j],
                                     dict(zip(keys, vals))))
        return fit_duration

    def _book_archive(self, job, r, ctx, start):
        """Per-sub-integration host bookkeeping (pptoas.py:567-792)."""
        quiet = ctx["quiet"]
        print_phase, print_flux = ctx["print_phase"], ctx["print_flux"]
        print_parangle = ctx["print_parangle"]
        addtnl_toa_flags = ctx["addtnl_toa_flags"]
        nu_ref_tuple = ctx["nu_ref_tuple"]
        d, datafile = job["d"], job["datafile"]
        nsub, nchan, nbin = job["nsub"], job["nchan"], job["nbin"]
        obs, nu_fits_a, nu_refs_a = job["obs"], job["nu_fits_a"], \
            job["nu_refs_a"]
        MJDs, DM0 = job["MJDs"], job["DM0"]
        ok_isubs, nok = job["ok_isubs"], job["nok"]
        models, model_index = job["models"], job["model_index"]
        mmean = None
        if ctx["print_flux"]:
            # the flux needs only each model row's mean: the scattered
            # model's mean is the unscattered one's (the scattering kernel's
            # zeroth harmonic is 1, pplib.py:4245-4260), so the reference's
            # per-sub-int rfft / irfft of the model (pptoas.py:628-636)
            # reduces to the row means, taken once per archive on the device
            mmean = models.mean(dim=-1).cpu().numpy() if isinstance(
                models, torch.Tensor) else np.asarray(models).mean(axis=-1)
        mask, flags_b = job["mask"], job["flags_b"]
        fit_duration = job["fit_duration"]
        batch_duration = r["batch_duration"]
        phis = np.zeros(nsub)
        phi_errs = np.zeros(nsub)
        TOAs = np.zeros(nsub, dtype="object")
        TOA_errs = np.zeros(nsub, dtype="object")
        DMs, DM_errs = np.zeros(nsub), np.zeros(nsub)
        GMs, GM_errs = np.zeros(nsub), np.zeros(nsub)
        taus, tau_errs = np.zeros(nsub), np.zeros(nsub)
        alphas, alpha_errs = np.zeros(nsub), np.zeros(nsub)
        scales = np.zeros([nsub, nchan])
        scale_errs = np.zeros([nsub, nchan])
        snrs = np.zeros(nsub)
        channel_snrs = np.zeros([nsub, nchan])
        profile_fluxes = np.zeros([nsub, nchan])
        profile_flux_errs = np.zeros([nsub, nchan])
        fluxes, flux_errs = np.zeros(nsub), np.zeros(nsub)
        flux_freqs = np.zeros(nsub)
        red_chi2s = np.zeros(nsub)
        covariances = np.zeros([nsub, self.nfit, self.nfit])
        nfevals = np.zeros(nsub, dtype="int")
        rcs = np.zeros(nsub, dtype="int")
        # ---- per-sub-integration bookkeeping (pptoas.py:567-711) -----
        uniform = (FAST_HOST and nok > 0 and
                   bool((flags_b == flags_b[0]).all()) and
                   int(np.count_nonzero(flags_b[0])) == self.nfit and
                   bool(mask.any(axis=1).all()))
        if uniform:
            fit_duration = self._book_uniform(job, r, ctx, fit_duration, dict(
                phis=phis, phi_errs=phi_errs, TOAs=TOAs, TOA_errs=TOA_errs,
                DMs=DMs, DM_errs=DM_errs, GMs=GMs, GM_errs=GM_errs, taus=taus,
                tau_errs=tau_errs, alphas=alphas, alpha_errs=alpha_errs,
                scales=scales, scale_errs=scale_errs, snrs=snrs,
                channel_snrs=channel_snrs, red_chi2s=red_chi2s,
                covariances=covariances, nfevals=nfevals, rcs=rcs,
                profile_fluxes=profile_fluxes,
                profile_flux_errs=profile_flux_errs, fluxes=fluxes,
                flux_errs=flux_errs, flux_freqs=flux_freqs, mmean=mmean))
        for j, isub in enumerate([] if uniform else ok_isubs):
            fit_flags_j = [int(v) for v in flags_b[j]]
            ok = mask[j].astype(bool)
            R = r["results"][j]
            status = int(R[_lib.RESULT_INDEX["status"]])
            _nu_zero_messages(fit_flags_j, nu_refs_a[isub])
            _raise_status(status)
            if (status & 0xff) not in (0, 1, 2, 4):
                _status_message(status & 0xff, datafile + "_%d" % isub)
            results = unpack_result(
                R, r["scales"][j][ok], r["scale_errs"][j][ok],
                r["channel_snrs"][j][ok], r["covariance"][j], fit_flags_j,
                batch_duration / nok)
            fit_duration += results.duration
            P = d.Ps[isub]
            epoch = d.epochs[isub]
            results.TOA = epoch + _MJD((results.phi * P + d.backend_delay)
                                       / (3600 * 24.))
            results.TOA_err = results.phi_err * P * 1e6
            if self.bary:
                df = d.doppler_factors[isub]
                if fit_flags_j[1]:
                    results.DM *= df
                if fit_flags_j[2]:
                    results.GM *= df ** 3
            else:
                df = 1.0
            freqsx = d.freqs[isub, ok]
            if print_flux:
                smm = mmean[model_index[j]][ok]
                profile_fluxes[isub, ok] = smm * results.scales
                profile_flux_errs[isub, ok] = abs(smm) * results.scale_errs
                flux, flux_err = weighted_mean(profile_fluxes[isub, ok],
                                               profile_flux_errs[isub, ok])
                flux_freq, _ = weighted_mean(freqsx,
                                             profile_flux_errs[isub, ok])
                fluxes[isub], flux_errs[isub] = flux, flux_err
                flux_freqs[isub] = flux_freq
            nu_refs_a[isub] = [results.nu_DM, results.nu_GM,
                               results.nu_tau]
            phis[isub], phi_errs[isub] = results.phi, results.phi_err
            TOAs[isub], TOA_errs[isub] = results.TOA, results.TOA_err
            DMs[isub], DM_errs[isub] = results.DM, results.DM_err
            GMs[isub], GM_errs[isub] = results.GM, results.GM_err
            taus[isub], tau_errs[isub] = results.tau, results.tau_err
            alphas[isub], alpha_errs[isub] = results.alpha, \
                results.alpha_err
            nfevals[isub], rcs[isub] = results.nfeval, results.return_code
            scales[isub, ok] = results.scales
            scale_errs[isub, ok] = results.scale_errs
            snrs[isub] = results.snr
            channel_snrs[isub, ok] = results.channel_snrs
            try:
                covariances[isub] = results.covariance_matrix
            except ValueError:
                ifit = np.where(fit_flags_j)[0]
                for ii, a in enumerate(ifit):
                    for jj, b in enumerate(ifit):
                        covariances[isub][a, b] = \
                            results.covariance_matrix[ii, jj]
            red_chi2s[isub] = results.red_chi2
            toa_flags = {}
            if not fit_flags_j[1]:
                results.DM = None
                results.DM_err = None
            if fit_flags_j[2]:
                toa_flags["gm"] = results.GM
                toa_flags["gm_err"] = results.GM_err
            if fit_flags_j[3]:
                if self.log10_tau:
                    toa_flags["scat_time"] = 10 ** results.tau * P / df * 1e6
                    toa_flags["log10_scat_time"] = results.tau + \
                        np.log10(P / df)
                    toa_flags["log10_scat_time_err"] = results.tau_err
                else:
                    toa_flags["scat_time"] = results.tau * P / df * 1e6
                    toa_flags["scat_time_err"] = results.tau_err * P / df \
                        * 1e6
                toa_flags["scat_ref_freq"] = results.nu_tau * df
                toa_flags["scat_ind"] = results.alpha
            if fit_flags_j[4]:
                toa_flags["scat_ind_err"] = results.alpha_err
            toa_flags["be"] = d.backend
            toa_flags["fe"] = d.frontend
            toa_flags["f"] = d.frontend + "_" + d.backend
            toa_flags["nbin"] = nbin
            toa_flags["nch"] = nchan
            toa_flags["nchx"] = len(freqsx)
            toa_flags["bw"] = freqsx.max() - freqsx.min()
            toa_flags["chbw"] = abs(d.bw) / nchan
            toa_flags["subint"] = isub
            toa_flags["tobs"] = d.subtimes[isub]
            toa_flags["fratio"] = freqsx.max() / freqsx.min()
            toa_flags["tmplt"] = self.modelfile
            toa_flags["snr"] = results.snr
            if nu_ref_tuple is not None and np.all(fit_flags_j[:2]):
                toa_flags["phi_DM_cov"] = results.covariance_matrix[0, 1]
            toa_flags["gof"] = results.red_chi2
            if print_phase:
                toa_flags["phs"] = results.phi
                toa_flags["phs_err"] = results.phi_err
            if print_flux:
                toa_flags["flux"] = fluxes[isub]
                toa_flags["flux_err"] = flux_errs[isub]
                toa_flags["flux_ref_freq"] = flux_freqs[isub]
            if print_parangle:
                toa_flags["par_angle"] = d.parallactic_angles[isub]
            for k, v in addtnl_toa_flags.items():
                toa_flags[k] = v
            self.TOA_list.append(TOA(datafile, results.nu_DM, results.TOA,
                                     results.TOA_err, d.telescope,
                                     d.telescope_code, results.DM,
                                     results.DM_err, toa_flags))
        # ---- DeltaDM (pptoas.py:713-729) ------------------------------
        DeltaDMs = DMs - DM0
        oks = np.asarray(d.ok_isubs)
        if np.all(DM_errs[oks]):
            DM_weights = DM_errs[oks] ** -2
        else:
            DM_weights = np.ones(len(DM_errs[oks]))
        DeltaDM_mean, DeltaDM_var = np.average(DeltaDMs[oks],
                                               weights=DM_weights,
                                               returned=True)
        DeltaDM_var = DeltaDM_var ** -1
        if len(oks) > 1:
            DeltaDM_var *= np.sum(((DeltaDMs[oks] - DeltaDM_mean) ** 2) *
                                  DM_weights) / (len(DeltaDMs[oks]) - 1)
        DeltaDM_err = DeltaDM_var ** 0.5
        self.order.append(datafile)
        self.obs.append(obs)
        self.doppler_fs.append(d.doppler_factors)
        self.nu0s.append(d.nu0)
        self.nu_fits.append(nu_fits_a)
        self.nu_refs.append(nu_refs_a)
        self.ok_isubs.append(d.ok_isubs)
        self.epochs.append(d.epochs)
        self.MJDs.append(MJDs)
        self.Ps.append(d.Ps)
        self.phis.append(phis)
        self.phi_errs.append(phi_errs)
        self.TOAs.append(TOAs)
        self.TOA_errs.append(TOA_errs)
        self.DM0s.append(DM0)
        self.DMs.append(DMs)
        self.DM_errs.append(DM_errs)
        self.DeltaDM_means.append(DeltaDM_mean)
        self.DeltaDM_errs.append(DeltaDM_err)
        self.GMs.append(GMs)
        self.GM_errs.append(GM_errs)
        self.taus.append(taus)
        self.tau_errs.append(tau_errs)
        self.alphas.append(alphas)
        self.alpha_errs.append(alpha_errs)
        self.scales.append(scales)
        self.scale_errs.append(scale_errs)
        self.snrs.append(snrs)
        self.channel_snrs.append(channel_snrs)
        self.profile_fluxes.append(profile_fluxes)
        self.profile_flux_errs.append(profile_flux_errs)
        self.fluxes.append(fluxes)
        self.flux_errs.append(flux_errs)
        self.flux_freqs.append(flux_freqs)
        self.covariances.append(covariances)
        self.red_chi2s.append(red_chi2s)
        self.nfevals.append(nfevals)
        self.rcs.append(rcs)
        self.fit_durations.append(fit_duration)
        if not quiet:
            print("--------------------------")
            print(datafile)
            print("~%.4f sec/TOA" % (fit_duration / len(d.ok_isubs)))
            print("Med. TOA error is %.3f us" % (np.median(
                phi_errs[oks]) * d.Ps.mean() * 1e6))
        tot_duration = time.time() - start
        if not quiet and len(self.ok_isubs):
            print("--------------------------")
            print("Total time: %.2f sec, ~%.4f sec/TOA" % (
                tot_duration,
                tot_duration / np.array(list(map(len, self.ok_isubs))
                                        ).sum()))

    def get_narrowband_TOAs(self, datafile=None, tscrunch=False,
                            fit_scat=False, log10_tau=True, scat_guess=None,
                            print_phase=False, print_flux=False,
                            print_parangle=False,
                            add_instrumental_response=False,
                            addtnl_toa_flags={}, method="trust-ncg",
                            bounds=None, show_plot=False, quiet=None):
        """pptoas.py:794-1189: one FFTFIT (fit_phase_shift, Ns=100) per usable
        channel of every sub-integration; all the channels of an archive are
        fitted in ONE batched device call (ppf_phase_shift_batch, the model
        row of each channel selected by index), then the reference's TOA
        bookkeeping per channel.  The reference's own fit_scat branch is
        unreachable (its rot_prof / nu_fit_tau are undefined there,
        pptoas.py:1001-1017); it raises here."""
        if quiet is None:
            quiet = self.quiet
        if fit_scat:
            raise NameError("name 'nu_fit_tau' is not defined "
                            "(pptoas.py:1002, the reference's narrowband "
                            "scattering branch is incomplete)")
        if add_instrumental_response and (self.ird["DM"] or
                                          len(self.ird["wids"])):
            raise NotImplementedError("instrumental response (SURVEY.md row "
                                      "19) is not on the accelerated path")
        print("You are using an experimental functionality of pptoas!")
        self._mcache = {}   # template portraits of this call (_models)
        self.nfit = 1
        self.fit_phi = True
        self.fit_tau = fit_scat
        self.fit_flags = [int(self.fit_phi), int(self.fit_tau)]
        self.log10_tau = log10_tau = False
        self.scat_guess = scat_guess
        start = time.time()
        datafiles = self.datafiles if datafile is None else [datafile]
        self.tscrunch = tscrunch
        self.add_instrumental_response = add_instrumental_response
        for iarch, datafile in enumerate(datafiles):
            fit_duration = 0.0
            try:
                data = load_data(datafile, dedisperse=False,
                                 dededisperse=False, tscrunch=tscrunch,
                                 pscrunch=True, fscrunch=False,
                                 rm_baseline=rm_baseline, flux_prof=False,
                                 refresh_arch=False, return_arch=False,
                                 quiet=quiet)
                if data.dmc:
                    if not quiet:
                        print("%s is dedispersed (dmc = 1).  Reloading it." %
                              datafile)
                    data = load_data(datafile, dedisperse=False,
                                     dededisperse=True, tscrunch=tscrunch,
                                     pscrunch=True, fscrunch=False,
                                     rm_baseline=rm_baseline,
                                     flux_prof=False, refresh_arch=False,
                                     return_arch=False, quiet=quiet)
                if not len(data.ok_isubs):
                    if not quiet:
                        print("No subints to fit for %s.  Skipping it." %
                              datafile)
                    continue
                self.ok_idatafiles.append(iarch)
            except RuntimeError:
                if not quiet:
                    print("Cannot load_data(%s).  Skipping it." % datafile)
                continue
            d = data
            nsub, nchan, nbin = d.nsub, d.nchan, d.nbin
            if d.source is None:
                d.source = "noname"
            obs = DataBunch(telescope=d.telescope, backend=d.backend,
                            frontend=d.frontend)
            phis = np.zeros([nsub, nchan])
            phi_errs = np.zeros([nsub, nchan])
            TOAs = np.zeros([nsub, nchan], dtype="object")
            TOA_errs = np.zeros([nsub, nchan], dtype="object")
            taus = np.zeros([nsub, nchan])
            tau_errs = np.zeros([nsub, nchan])
            scales = np.zeros([nsub, nchan])
            scale_errs = np.zeros([nsub, nchan])
            channel_snrs = np.zeros([nsub, nchan])
            profile_fluxes = np.zeros([nsub, nchan])
            profile_flux_errs = np.zeros([nsub, nchan])
            channel_red_chi2s = np.zeros([nsub, nchan])
            covariances = np.zeros([nsub, nchan, self.nfit, self.nfit])
            nfevals = np.zeros([nsub, nchan], dtype="int")
            rcs = np.zeros([nsub, nchan], dtype="int")
            MJDs = np.array([d.epochs[isub].in_days() for isub in range(nsub)],
                            dtype=np.double)
            ok_isubs = list(d.ok_isubs)
            models, model_index = self._models(d, ok_isubs, False, quiet)
            # every (sub-int, usable channel) row of the archive
            rows_s, rows_c, midx = [], [], []
            for j, isub in enumerate(ok_isubs):
                for ichan in d.ok_ichans[isub]:
                    rows_s.append(isub)
                    rows_c.append(int(ichan))
                    midx.append(model_index[j] * nchan + int(ichan))
            rows_s = np.array(rows_s, dtype=int)
            rows_c = np.array(rows_c, dtype=int)
            t_fit = time.time()
            out = np.zeros((0, 8))
            if len(rows_s):
                prof = np.asarray(d.subints)[rows_s, 0, rows_c]
                p32 = prof.astype(np.float32)
                if np.array_equal(p32.astype(np.float64), prof):
                    prof = p32
                errs = np.asarray(d.noise_stds)[rows_s, 0, rows_c]
                out = engine.phase_shift_batch(
                    prof, models.reshape(-1, nbin), errs, Ns=100,
                    bounds=(-0.5, 0.5),
                    model_index=np.array(midx, dtype=np.int32)).cpu().numpy()
            per = (time.time() - t_fit) / max(1, len(rows_s))
            for r, (isub, ichan) in enumerate(zip(rows_s, rows_c)):
                phase, phase_err, scale, scale_err, snr, red_chi2 = out[r, :6]
                fit_duration += per
                P = d.Ps[isub]
                epoch = d.epochs[isub]
                TOA_r = epoch + _MJD((phase * P + d.backend_delay) /
                                     (3600 * 24.))
                TOA_err = phase_err * P * 1e6
                if print_flux:
                    model_prof = models[model_index[ok_isubs.index(isub)]][
                        ichan]
                    smm = np.copy(model_prof).mean()
                    profile_fluxes[isub, ichan] = smm * scale
                    profile_flux_errs[isub, ichan] = abs(smm) * scale_err
                phis[isub, ichan] = phase
                phi_errs[isub, ichan] = phase_err
                TOAs[isub, ichan] = TOA_r
                TOA_errs[isub, ichan] = TOA_err
                scales[isub, ichan] = scale
                scale_errs[isub, ichan] = scale_err
                channel_snrs[isub, ichan] = snr
                channel_red_chi2s[isub] = red_chi2     # (sic) pptoas.py:1094
                toa_flags = {}
                toa_flags["be"] = d.backend
                toa_flags["fe"] = d.frontend
                toa_flags["f"] = d.frontend + "_" + d.backend
                toa_flags["nbin"] = nbin
                toa_flags["bw"] = abs(d.bw) / nchan
                toa_flags["subint"] = isub
                toa_flags["chan"] = ichan
                toa_flags["tobs"] = d.subtimes[isub]
                toa_flags["tmplt"] = self.modelfile
                toa_flags["snr"] = snr
                toa_flags["gof"] = red_chi2
                if print_phase:
                    # the reference reads results.phi, which fit_phase_shift
                    # does not return (pptoas.py:1120)
                    raise AttributeError("'DataBunch' object has no "
                                         "attribute 'phi'")
                if print_flux:
                    # the reference reads fluxes[isub], never defined on this
                    # path (pptoas.py:1123)
                    raise NameError("name 'fluxes' is not defined")
                if print_parangle:
                    toa_flags["par_angle"] = d.parallactic_angles[isub]
                for k, v in addtnl_toa_flags.items():
                    toa_flags[k] = v
                self.TOA_list.append(TOA(datafile, d.freqs[isub, ichan],
                                         TOA_r, TOA_err, d.telescope,
                                         d.telescope_code, None, None,
                                         toa_flags))
            self.order.append(datafile)
            self.obs.append(obs)
            self.doppler_fs.append(d.doppler_factors)
            self.ok_isubs.append(d.ok_isubs)
            self.epochs.append(d.epochs)
            self.MJDs.append(MJDs)
            self.Ps.append(d.Ps)
            self.phis.append(phis)
            self.phi_errs.append(phi_errs)
            self.TOAs.append(TOAs)
            self.TOA_errs.append(TOA_errs)
            self.taus.append(taus)
            self.tau_errs.append(tau_errs)
            self.scales.append(scales)
            self.scale_errs.append(scale_errs)
            self.channel_snrs.append(channel_snrs)
            self.profile_fluxes.append(profile_fluxes)
            self.profile_flux_errs.append(profile_flux_errs)
            self.covariances.append(covariances)
            self.channel_red_chi2s.append(channel_red_chi2s)
            self.nfevals.append(nfevals)
            self.rcs.append(rcs)
            self.fit_durations.append(fit_duration)
            if not quiet:
                print("--------------------------")
                print(datafile)
                print("~%.4f sec/TOA" % (fit_duration / len(self.TOA_list)))
                print("Med. TOA error is %.3f us" % (np.median(
                    phi_errs[d.ok_isubs]) * d.Ps.mean() * 1e6))
        tot_duration = time.time() - start
        if not quiet and len(self.ok_isubs):
            print("--------------------------")
            print("Total time: %.2f sec, ~%.4f sec/TOA" % (
                tot_duration, tot_duration / len(self.TOA_list)))

    # ------------------------------------------------------------------
    # fit inspection and channel zapping (pptoas.py:1266-1480)
    # ------------------------------------------------------------------
    def _load_fit_data(self, datafile, quiet):
        """show_fit's reload of the archive (pptoas.py:1393-1409)."""
        kw = dict(dedisperse=False, dededisperse=False,
                  tscrunch=getattr(self, "tscrunch", False), pscrunch=True,
                  fscrunch=False, rm_baseline=True, flux_prof=False,
                  refresh_arch=False, return_arch=False, quiet=quiet)
        data = load_data(datafile, **kw)
        if data.dmc:
            if not quiet:
                print("%s is dedispersed (dmc = 1).  Reloading it." %
                      datafile)
            kw["dededisperse"] = True
            data = load_data(datafile, **kw)
        return data

    def _fit_model(self, data, ifile, isub, quiet, cache=None):
        """The unscaled (scattered) model portrait of show_fit
        (pptoas.py:1415-1459) for one sub-integration.  Un-scattered models
        depend only on the channel frequencies and are cached per archive."""
        if self.is_FITS_model:
            raise NotImplementedError("FITS (archive) templates need PSRCHIVE")
        if self.add_instrumental_response and \
                (self.ird["DM"] or len(self.ird["wids"])):
            raise NotImplementedError("instrumental response (SURVEY.md row "
                                      "19) is not on the accelerated path")
        freqs = data.freqs[isub]
        tau = self.taus[ifile][isub]
        key = freqs.tobytes()
        if tau == 0.0 and cache is not None and key in cache:
            return cache[key]
        model_name, ngauss, model = read_model(
            self.modelfile, data.phases, freqs, data.Ps.mean(), quiet=quiet)
        if tau != 0.0:
            (model_name, model_code, model_nu_ref, ngauss, gparams, _mff,
             _ma, _mfa) = read_model(self.modelfile, quiet=quiet)
            if self.log10_tau:
                tau = 10 ** tau
            nu_ref_tau = self.nu_refs[ifile][isub][2]
            alpha = self.alphas[ifile][isub]
            # the reference convolves the un-scattered portrait with the
            # fitted scattering kernel on the host, irfft(B(tau (nu /
            # nu_ref_tau)^alpha) rfft(model)) (pptoas.py:1455-1459); the same
            # portrait is gen_gaussian_portrait's own scattered branch
            # (pplib.py:948-953) with tau at the model's reference frequency,
            # built on the device (k_gauss_port: one LDS FFT per channel)
            gparams = np.copy(gparams)
            gparams[1] = tau * data.nbin * (model_nu_ref / nu_ref_tau) ** alpha
            model = gen_gaussian_portrait(model_code, gparams, alpha,
                                          data.phases, freqs, model_nu_ref)
        elif cache is not None:
            cache[key] = (model_name, model)
        return model_name, model

    def _fit_phases(self, data, ifile, isub):
        """Per-channel rotation of show_fit's rotate_portrait_full call
        (pptoas.py:1410-1418, 1460-1461): fitted phi, DM, GM (Doppler
        corrected back to the topocentric values) at the output ν_refs."""
        phi = self.phis[ifile][isub]
        DM = self.DMs[ifile][isub]
        GM = self.GMs[ifile][isub]
        if self.bary:
            DM /= self.doppler_fs[ifile][isub]
            GM /= self.doppler_fs[ifile][isub] ** 3
        nu_ref_DM, nu_ref_GM, _ = self.nu_refs[ifile][isub]
        return _pptl.phase_shifts(phi, DM, GM, data.freqs[isub], nu_ref_DM,
                                  nu_ref_GM, data.Ps[isub], False)

    def show_fit(self, datafile=None, isub=0, rotate=0.0, show=True,
                 return_fit=False, savefig=False, quiet=None):
        """pptoas.py:1375-1480: the rotated data portrait and the scaled
        fitted model of one sub-integration (rotation on the GPU).  The plot
        itself is outside the accelerated path: show=True raises."""
        if quiet is None:
            quiet = self.quiet
        if show:
            raise NotImplementedError("plotting is outside the accelerated "
                                      "path (SURVEY.md section 2, row 20)")
        if datafile is None:
            datafile = self.datafiles[0]
        ifile = list(np.array(self.datafiles)[self.ok_idatafiles]).index(
            datafile)
        data = self._load_fit_data(datafile, quiet)
        model_name, model = self._fit_model(data, ifile, isub, quiet)
        ph = self._fit_phases(data, ifile, isub)
        port = engine.rotate_rows(np.asarray(data.subints[isub, 0]),
                                  ph).cpu().numpy()
        if rotate:
            model = _pplib.rotate_data(model, rotate)
            port = _pplib.rotate_data(port, rotate)
        if data.masks is not None:
            port *= data.masks[isub, 0]
        model_scaled = np.transpose(self.scales[ifile][isub] *
                                    np.transpose(model))
        if return_fit:
            return (port, model_scaled, data.ok_ichans[isub],
                    data.freqs[isub], data.noise_stds[isub, 0])

    def get_channels_to_zap(self, SNR_threshold=8.0, rchi2_threshold=1.3,
                            iterate=True, show=False):
        """pptoas.py:1266-1343.  NB: get_TOAs(...) needs to have been called
        first.  Per archive, the reduced chi^2 of every usable channel of
        every fitted sub-integration (show_fit + get_red_chi2 with
        dof = nbin - 2, pplib.py:754-779) is ONE batched device call
        (ppf_resid_chi2_batch: rotate, subtract the scaled model, reduce);
        the S/N / chi^2 selection that follows is the reference's host logic.
        Fills self.channel_red_chi2s and self.zap_channels."""
        if show:
            raise NotImplementedError("plotting is outside the accelerated "
                                      "path (SURVEY.md section 2, row 20)")
        for iarch, ok_idatafile in enumerate(self.ok_idatafiles):
            datafile = self.datafiles[ok_idatafile]
            data = self._load_fit_data(datafile, True)
            nbin = data.nbin
            isubs = list(self.ok_isubs[iarch])
            cache, slots, models, rows, phases, midx, scl, errs, chans = \
                {}, {}, [], [], [], [], [], [], []
            for isub in isubs:
                ok = np.asarray(data.ok_ichans[isub], dtype=int)
                _, model = self._fit_model(data, iarch, isub, True, cache)
                port = np.asarray(data.subints[isub, 0])[ok]
                if data.masks is not None:
                    m = np.asarray(data.masks[isub, 0])[ok]
                    if not np.all(m == 1.0):
                        port = port * m
                rows.append(port)
                phases.append(self._fit_phases(data, iarch, isub)[ok])
                slot = slots.setdefault(id(model), len(models))
                if slot == len(models):
                    models.append(model)
                midx.append(slot * data.nchan + ok)
                scl.append(np.asarray(self.scales[iarch][isub])[ok])
                errs.append(np.asarray(data.noise_stds[isub, 0])[ok])
                chans.append(ok)
            if len(isubs):
                rows_a = np.concatenate(rows)
                r32 = rows_a.astype(np.float32)
                if np.array_equal(r32.astype(np.float64), rows_a):
                    rows_a = r32          # PSRCHIVE amplitudes are float32
                chi2 = engine.resid_chi2_rows(
                    rows_a, np.concatenate(phases),
                    np.concatenate(models).reshape(-1, nbin),
                    np.concatenate(midx), np.concatenate(scl),
                    np.concatenate(errs), nbin - 2).cpu().numpy()
            channel_red_chi2s, zap_channels = [], []
            pos = 0
            for j, isub in enumerate(isubs):
                ok_ichans = chans[j]
                red_chi2s = list(chi2[pos:pos + len(ok_ichans)])
                pos += len(ok_ichans)
                channel_snrs = self.channel_snrs[iarch][isub]
                channel_red_chi2s.append(red_chi2s)
                zap_channels.append(_select_zap(
                    red_chi2s, ok_ichans, channel_snrs, SNR_threshold,
                    rchi2_threshold, iterate))
            self.channel_red_chi2s.append(channel_red_chi2s)
            self.zap_channels.append(zap_channels)


def _select_zap(red_chi2s, ok_ichans, channel_snrs, SNR_threshold,
                rchi2_threshold, iterate):
    """The channel selection of pptoas.py:1296-1333 for one sub-integration:
    chi^2 above threshold or NaN, or channel S/N below
    (SNR_threshold^2 / nchx)^0.5; with iterate, the S/N threshold is raised
    as channels are removed until nothing new is cut."""
    nchx = len(ok_ichans)
    bad = []
    threshold = (SNR_threshold ** 2.0 / nchx) ** 0.5 if nchx else np.inf
    for ok_ichan, rchi2 in zip(ok_ichans, red_chi2s):
        if rchi2 > rchi2_threshold:
            bad.append(ok_ichan)
        elif np.isnan(rchi2):
            bad.append(ok_ichan)
        elif SNR_threshold and channel_snrs[ok_ichan] < threshold:
            bad.append(ok_ichan)
    if iterate and SNR_threshold and len(bad):
        old_len = len(bad)
        added_new = True
        while added_new and (nchx - len(bad)):
            threshold = (SNR_threshold ** 2.0 / (nchx - len(bad))) ** 0.5
            bad_set = set(int(b) for b in bad)
            for ok_ichan in ok_ichans:
                if int(ok_ichan) in bad_set:
                    continue
                if channel_snrs[ok_ichan] < threshold:
                    bad.append(ok_ichan)
                    bad_set.add(int(ok_ichan))
            added_new = bool(len(bad) - old_len)
            old_len = len(bad)
    return bad

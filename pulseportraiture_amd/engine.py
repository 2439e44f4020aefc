"""Batched device engine: torch tensors in, libppfit kernels, torch tensors out.

PyTorch supplies device memory, the current HIP stream and (in dist.py) the
RCCL communicator; all arithmetic happens in libppfit's HIP kernels.  Every
function here accepts numpy arrays or torch tensors (host or device) and
returns device tensors; the drop-in modules (pplib / pptoaslib / pptoas)
convert to the reference's numpy/DataBunch forms.
"""
import ctypes
import os
import threading
import warnings

import numpy as np
import torch

from . import _lib
from .timeline import span

DEVICE_TYPE = "cuda"   # torch's name for HIP devices on ROCm


def device(dev=None):
    if not torch.cuda.is_available():
        raise RuntimeError("pulseportraiture_amd needs a HIP device "
                           "(torch.cuda.is_available() is False); there is "
                           "no CPU fallback")
    if dev is None:
        return torch.device(DEVICE_TYPE, torch.cuda.current_device())
    dev = torch.device(dev)
    if dev.type != DEVICE_TYPE:
        raise ValueError("device must be a HIP device, got %s" % dev)
    return dev if dev.index is not None else torch.device(
        DEVICE_TYPE, torch.cuda.current_device())


def to_dev(x, dev, dtype):
    """Contiguous device tensor of dtype (None passes through)."""
    if x is None:
        return None
    if isinstance(x, torch.Tensor):
        return x.to(device=dev, dtype=dtype).contiguous()
    a = np.ascontiguousarray(x)
    if not a.flags.writeable:
        # the host array is only read (copied to the device): torch's
        # warning about non-writable NumPy memory does not apply
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", UserWarning)
            return torch.as_tensor(a, dtype=dtype).to(dev)
    return torch.as_tensor(a, dtype=dtype).to(dev)


_PIN = {}
_PIN_LOCK = threading.Lock()


def _pinned(tag, nbytes):
    """A page-locked staging buffer of at least nbytes, one per (thread,
    tag), grown on demand and reused: the single-call APIs copy their host
    arrays through it instead of torch's pageable path (whose per-call
    staging made a 512 x 2048 rotate_data take 1.6-25 ms)."""
    key = (threading.get_ident(), tag)
    with _PIN_LOCK:
        buf = _PIN.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8,
                              pin_memory=True)
            _PIN[key] = buf
    return buf


_STAGE = threading.local()
# fit inputs staged by ppf_copy_from_pinned's kernel (1) or a copy-engine
# transfer (0); env PPF_STAGE_KERNEL
_STAGE_KERNEL = os.environ.get("PPF_STAGE_KERNEL", "1") != "0"
_NPD = {torch.float64: np.float64, torch.float32: np.float32,
        torch.int32: np.int32, torch.uint8: np.uint8}


def _stage_host(items, dev):
    """[(host array, torch dtype)] -> device tensors of the same shapes:
    the arrays are packed (256-B aligned) into one of the calling thread's
    two page-locked buffers and copied with ONE non-blocking copy on the
    current stream; a buffer is refilled only after the copy that last
    read it has completed (its event)."""
    arrs = [np.ascontiguousarray(x, dtype=_NPD[dt]) for x, dt in items]
    offs, o = [], 0
    for a in arrs:
        offs.append(o)
        o += -(-a.nbytes // 256) * 256
    total = max(o, 256)
    ring = getattr(_STAGE, "ring", None)
    if ring is None:
        ring = _STAGE.ring = [[[None, None], [None, None]], 0]
    slot = ring[0][ring[1] % 2]
    ring[1] += 1
    if slot[1] is not None:
        slot[1].synchronize()
    if slot[0] is None or slot[0].numel() < total:
        slot[0] = torch.empty(max(total, 1 << 20), dtype=torch.uint8,
                              pin_memory=True)
    hb = slot[0].numpy()
    for a, off in zip(arrs, offs):
        hb[off:off + a.nbytes] = a.reshape(-1).view(np.uint8)
    d = torch.empty(total, dtype=torch.uint8, device=dev)
    global _STAGE_KERNEL
    staged = False
    if _STAGE_KERNEL:
        # read by a kernel over PCIe: no copy-engine transfer, so it never
        # queues behind an archive upload (ppf_copy_from_pinned).  A pinned
        # buffer the device cannot map (host-registered without the mapped
        # flag, another allocator) makes the call return an error: then the
        # copy engine takes this and every later staging of the process
        ctx = _lib.context(dev.index)
        rc = _lib.load().ppf_copy_from_pinned(
            ctx, _p(d), ctypes.c_void_p(slot[0].data_ptr()), total,
            _stream(dev))
        if rc == 0:
            staged = True
        else:
            _STAGE_KERNEL = False
    if not staged:
        d.copy_(slot[0][:total], non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    slot[1] = ev
    return [d[off:off + a.nbytes].view(dt).view(a.shape)
            for a, (_, dt), off in zip(arrs, items, offs)]


def host_to_dev(x, dev, dtype):
    """to_dev through the caller's pinned staging buffer (the copy is
    ordered on the current stream; the buffer is reused only by the same
    thread's next call, which comes after this call's own synchronising
    read-back)."""
    a = np.ascontiguousarray(x)
    t = torch.as_tensor(a) if a.flags.writeable else torch.from_numpy(a.copy())
    t = t.to(dtype)
    buf = _pinned("in", t.numel() * t.element_size())
    h = buf[:t.numel() * t.element_size()].view(t.dtype).view(t.shape)
    h.copy_(t)
    return h.to(dev, non_blocking=True)


def dev_to_host(t):
    """A NumPy copy of device tensor t, read back through the caller's
    pinned staging buffer (synchronises the current stream)."""
    n = t.numel() * t.element_size()
    buf = _pinned("out", n)
    h = buf[:n].view(t.dtype).view(t.shape)
    h.copy_(t, non_blocking=True)
    torch.cuda.current_stream(t.device).synchronize()
    return h.numpy().copy()


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _data_dtype(x):
    if isinstance(x, torch.Tensor):
        return torch.float32 if x.dtype == torch.float32 else torch.float64
    return torch.float32 if np.asarray(x).dtype == np.float32 else \
        torch.float64


def _host(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def x_subints(fit_flags, init, log10_tau, nsub):
    """Sub-ints whose fit streams the cross spectrum X (k_classify's test,
    restated on the host): scattering flags set, or a nonzero initial tau
    (10**tau with log10_tau, pptoaslib.py:271-276)."""
    fl = _host(fit_flags).reshape(-1, 5)
    if fl.shape[0] == 1:
        fl = np.repeat(fl, nsub, axis=0)
    x3 = _host(init).reshape(nsub, 5)[:, 3]
    with np.errstate(over="ignore"):
        tau0 = 10.0 ** x3 if log10_tau else x3
    return int(np.count_nonzero((fl[:, 3] != 0) | (fl[:, 4] != 0) |
                                (tau0 != 0.0)))


SOLVER = os.environ.get("PPF_SOLVER", "newton")
# phase/DM/GM moments: None = the library's choice (from the stored cross
# spectrum where the GetTOAs guess rides along in the spectrum pass), True /
# False = always from X / always from the fused k_xmom_g pass (env PPF_MOM_X
# = 1 / 0)
MOM_X = {"1": True, "0": False}.get(os.environ.get("PPF_MOM_X", ""), None)


def _solver(name):
    name = SOLVER if name is None else name
    if name not in ("newton", "scipy"):
        raise ValueError("solver must be 'newton' or 'scipy', not %r" % name)
    return name


def fit_batch(data, model, freqs, P, init, fit_flags, nu_fits=None,
              nu_outs=None, errs=None, chan_mask=None, model_index=None,
              log10_tau=False, option=0, is_toa=True, mode=_lib.PPF_MODE_FULL,
              max_iter=0, guess=False, guess_weights=None, guess_DM=None,
              guess_Ns=100, guess_tau=None, dev=None, workspace=None,
              n_x=None, no_hcut=False, max_workspace=None, guess_ref=0,
              bounds=None, solver=None, mom_x=None, spin_wait=False):
    """Fit nsub sub-integrations: data [nsub, nchan, nbin] (f32 or f64),
    model [nmodel, nchan, nbin] (or [nchan, nbin]), freqs [nsub, nchan],
    P [nsub], init [nsub, 5], fit_flags [nsub, 5] (or [5]).

    n_x: cross-spectrum slots (sub-ints whose fit streams X); None computes
    it from fit_flags / init (x_subints).  no_hcut: sum every harmonic
    (PPF_OPT_NO_HCUT).  guess_ref: frame of the guess profile (0: mean
    frequency then phase_transform to nu_fit, GetTOAs; 1: nu_fit, ppalign).
    bounds: method='TNC' box, [5, 2] or [nsub, 5, 2] (lower, upper; None or
    NaN = unbounded), or None for an unbounded fit.
    solver: minimiser of the unbounded fits, "newton" (scaled Newton trust
    region with an exact subproblem: the same stationary point, in 3x fewer
    passes over the cross spectrum for scattering fits and half the data
    passes for ppalign's) or "scipy" (scipy trust-ncg's own path,
    PPF_OPT_SCIPY_TR); None = SOLVER (env PPF_SOLVER, default "newton").
    mom_x: take the moments of the phase/DM/GM fits from the stored cross
    spectrum (True, PPF_OPT_MOM_X) or from the fused pass (False,
    PPF_OPT_FUSED_MOM); None = MOM_X (env PPF_MOM_X; unset: the library
    chooses).
    spin_wait: poll the read-backs of the iteration loop on the host
    (PPF_OPT_SPIN_WAIT) -- for callers with no host threads of their own.
    max_workspace: workspace budget in bytes (default
    half the free device memory); a batch needing more is fitted in
    consecutive chunks of sub-ints (a sub-int's result does not depend on
    the batch it is in).

    Returns a dict of device tensors: results [nsub, 32] (see
    _lib.RESULT_INDEX), scales/scale_errs/channel_snrs [nsub, nchan],
    covariance [nsub, 5, 5], and the workspace (reusable)."""
    dev = device(dev)
    f64 = torch.float64
    if n_x is None and not isinstance(init, torch.Tensor) and \
            not isinstance(fit_flags, torch.Tensor):
        # counted from the host arrays before the upload (no device
        # round trip)
        n_x = x_subints(fit_flags, init, log10_tau,
                        int(np.asarray(init).size // 5))
    data_t = to_dev(data, dev, _data_dtype(data))
    if data_t.dim() != 3:
        raise ValueError("data must be [nsub, nchan, nbin]")
    nsub, nchan, nbin = data_t.shape
    # the per-sub-int inputs that arrive as host arrays travel in ONE pinned
    # buffer and ONE asynchronous copy on the current stream (a pageable
    # copy per input synchronises the host each time and queues behind any
    # archive upload on the copy engine: GetTOAs' fit worker measured
    # ~7.7 ms per 64-sub-int archive that way)
    specs = [("freqs", freqs, f64), ("P", P, f64), ("init", init, f64),
             ("flags", fit_flags, torch.int32), ("nu_fits", nu_fits, f64),
             ("nu_outs", nu_outs, f64), ("errs", errs, f64),
             ("mask", chan_mask, torch.uint8), ("mi", model_index, torch.int32)]
    if guess:
        specs += [("gtau", guess_tau, f64), ("gw", guess_weights, f64),
                  ("gdm", guess_DM, f64)]
    host = [(k, x, dt) for k, x, dt in specs
            if x is not None and not isinstance(x, torch.Tensor)]
    if host:
        with span("fit.stage"):
            up = dict(zip([k for k, _, _ in host], _stage_host(
                [(x, dt) for _, x, dt in host], dev)))
        freqs, P, init = up.get("freqs", freqs), up.get("P", P), \
            up.get("init", init)
        fit_flags, nu_fits = up.get("flags", fit_flags), \
            up.get("nu_fits", nu_fits)
        nu_outs, errs = up.get("nu_outs", nu_outs), up.get("errs", errs)
        chan_mask, model_index = up.get("mask", chan_mask), \
            up.get("mi", model_index)
        guess_tau, guess_weights = up.get("gtau", guess_tau), \
            up.get("gw", guess_weights)
        guess_DM = up.get("gdm", guess_DM)
    model_t = to_dev(model, dev, f64)
    if model_t.dim() == 2:
        model_t = model_t.unsqueeze(0)
    if model_t.shape[1:] != (nchan, nbin):
        raise ValueError("model shape %s != [*, %d, %d]" %
                         (tuple(model_t.shape), nchan, nbin))
    freqs_t = to_dev(freqs, dev, f64).reshape(-1)
    if freqs_t.numel() == nchan:
        freqs_t = freqs_t.repeat(nsub)
    freqs_t = freqs_t.reshape(nsub, nchan).contiguous()
    P_t = to_dev(P, dev, f64).reshape(-1)
    if P_t.numel() == 1:
        P_t = P_t.repeat(nsub)
    init_t = to_dev(init, dev, f64).reshape(nsub, 5).contiguous()
    flags_t = to_dev(fit_flags, dev, torch.int32).reshape(-1)
    if flags_t.numel() == 5:
        flags_t = flags_t.repeat(nsub)
    flags_t = flags_t.reshape(nsub, 5).contiguous()
    def nan3():
        return torch.full((nsub, 3), float("nan"), dtype=f64, device=dev)
    nu_fits_t = nan3() if nu_fits is None else \
        to_dev(nu_fits, dev, f64).reshape(nsub, 3).contiguous()
    nu_outs_t = nan3() if nu_outs is None else \
        to_dev(nu_outs, dev, f64).reshape(nsub, 3).contiguous()
    errs_t = None if errs is None else \
        to_dev(errs, dev, f64).reshape(nsub, nchan).contiguous()
    mask_t = None if chan_mask is None else \
        to_dev(chan_mask, dev, torch.uint8).reshape(nsub, nchan).contiguous()
    mi_t = None if model_index is None else \
        to_dev(model_index, dev, torch.int32).reshape(nsub).contiguous()
    gw_t = gdm_t = gtau_t = None
    if guess:
        if guess_tau is not None:
            gtau_t = to_dev(guess_tau, dev, f64).reshape(-1)
            if gtau_t.numel() == 1:
                gtau_t = gtau_t.repeat(nsub)
        gw_t = to_dev(guess_weights, dev, f64).reshape(nsub, nchan).contiguous()
        gdm_t = to_dev(guess_DM, dev, f64).reshape(-1)
        if gdm_t.numel() == 1:
            gdm_t = gdm_t.repeat(nsub)
    bnd_t = None
    if bounds is not None:
        b = np.array([[np.nan if v is None else float(v) for v in lu]
                      for lu in np.asarray(bounds, dtype=object).reshape(-1, 2)
                      ], dtype=float).reshape(-1, 5, 2)
        if b.shape[0] == 1:
            b = np.repeat(b, nsub, axis=0)
        bnd_t = to_dev(b.reshape(nsub, 5, 2), dev, f64)
    per_sub = dict(data=data_t, freqs=freqs_t, P=P_t, init=init_t,
                   flags=flags_t, nu_fits=nu_fits_t, nu_outs=nu_outs_t,
                   errs=errs_t, mask=mask_t, mi=mi_t, gw=gw_t, gdm=gdm_t,
                   gtau=gtau_t, bounds=bnd_t)
    if n_x is None:
        n_x = x_subints(flags_t, init_t, log10_tau, nsub)
    xsel = None
    cfg = dict(model=model_t, log10_tau=log10_tau, option=option,
               is_toa=is_toa, mode=mode, max_iter=max_iter, guess=guess,
               guess_Ns=guess_Ns, no_hcut=no_hcut, guess_ref=guess_ref,
               solver=_solver(solver),
               mom_x=MOM_X if mom_x is None else bool(mom_x),
               spin_wait=bool(spin_wait))
    lib = _lib.load()
    d0 = _desc(per_sub, 0, nsub, n_x, cfg)
    need = _desc_workspace_bytes(lib, d0)
    if max_workspace is None and (need <= (64 << 20) or nsub == 1):
        # small batches (the single-call APIs) skip the free-memory query
        return _fit_slice(lib, dev, per_sub, 0, nsub, n_x, cfg, workspace,
                          d0, need)
    if max_workspace is None:
        free, _ = torch.cuda.mem_get_info(dev)
        max_workspace = free // 2
    if need <= max_workspace:
        return _fit_slice(lib, dev, per_sub, 0, nsub, n_x, cfg, workspace,
                          d0, need)
    # chunks of equal size whose workspace fits the budget
    per = max(1, int(nsub * max_workspace // max(need, 1)))
    while per > 1 and _workspace_bytes(lib, per_sub, 0, per, per, cfg) > \
            max_workspace:
        per //= 2
    if xsel is None:
        fl = _host(flags_t)
        x3 = _host(init_t)[:, 3]
        with np.errstate(over="ignore"):
            tau0 = 10.0 ** x3 if log10_tau else x3
        xsel = (fl[:, 3] != 0) | (fl[:, 4] != 0) | (tau0 != 0.0)
    outs, ws = [], None
    for c0 in range(0, nsub, per):
        c1 = min(nsub, c0 + per)
        r = _fit_slice(lib, dev, per_sub, c0, c1,
                       int(np.count_nonzero(xsel[c0:c1])), cfg, ws)
        ws = r["workspace"]
        outs.append(r)
    out = {k: torch.cat([o[k] for o in outs], 0)
           for k in ("results", "scales", "scale_errs", "channel_snrs",
                     "covariance")}
    out["workspace"] = ws
    out["_keep"] = tuple(o["_keep"] for o in outs)
    return out


def _desc(per_sub, c0, c1, n_x, cfg):
    """ppf_fit_desc of sub-ints [c0, c1) (pointers into the device tensors;
    outputs left NULL)."""
    sl = slice(c0, c1)

    def pp(t):
        return None if t is None else _p(t[sl])
    data_t = per_sub["data"]
    nchan, nbin = data_t.shape[1:]
    model_t = cfg["model"]
    d = _lib.FitDesc()
    d.nsub, d.nchan, d.nbin = c1 - c0, nchan, nbin
    d.data_dtype = _lib.PPF_F32 if data_t.dtype == torch.float32 else \
        _lib.PPF_F64
    d.data, d.model, d.nmodel = pp(data_t), _p(model_t), model_t.shape[0]
    d.model_index, d.chan_mask = pp(per_sub["mi"]), pp(per_sub["mask"])
    d.freqs, d.P, d.errs = pp(per_sub["freqs"]), pp(per_sub["P"]), \
        pp(per_sub["errs"])
    d.init, d.fit_flags = pp(per_sub["init"]), pp(per_sub["flags"])
    d.nu_fits, d.nu_outs = pp(per_sub["nu_fits"]), pp(per_sub["nu_outs"])
    d.log10_tau, d.option = int(bool(cfg["log10_tau"])), int(cfg["option"])
    d.is_toa = int(bool(cfg["is_toa"]))
    d.mode, d.max_iter = int(cfg["mode"]), int(cfg["max_iter"])
    d.guess, d.guess_Ns = int(bool(cfg["guess"])), int(cfg["guess_Ns"])
    d.guess_weights, d.guess_DM = pp(per_sub["gw"]), pp(per_sub["gdm"])
    d.guess_tau = pp(per_sub["gtau"])
    d.x_subints = int(max(n_x, 1)) if n_x < (c1 - c0) else 0
    d.options = (_lib.OPT_NO_HCUT if cfg["no_hcut"] else 0) | \
        (_lib.OPT_NO_X if n_x == 0 else 0) | \
        (_lib.OPT_SCIPY_TR if cfg.get("solver") == "scipy" else 0) | \
        (_lib.OPT_MOM_X if cfg.get("mom_x") is True else 0) | \
        (_lib.OPT_FUSED_MOM if cfg.get("mom_x") is False else 0) | \
        (_lib.OPT_SPIN_WAIT if cfg.get("spin_wait") else 0)
    d.guess_ref = int(cfg["guess_ref"])
    d.bounds = pp(per_sub["bounds"])
    return d


def _workspace_bytes(lib, per_sub, c0, c1, n_x, cfg):
    return _desc_workspace_bytes(lib, _desc(per_sub, c0, c1, n_x, cfg))


def _desc_workspace_bytes(lib, d):
    nbytes = lib.ppf_fit_workspace_bytes(ctypes.byref(d))
    if nbytes == 0:
        raise NotImplementedError(
            "unsupported shape nsub=%d nchan=%d nbin=%d (nbin must be even in"
            " [32, 8192] or odd in [33, 4095]; longer rows fit without the"
            " GetTOAs guess, up to 2^23 transform points)" %
            (d.nsub, d.nchan, d.nbin))
    return nbytes


def _fit_slice(lib, dev, per_sub, c0, c1, n_x, cfg, workspace, d=None,
               nbytes=None):
    """ppf_fit_batch over sub-ints [c0, c1) (d / nbytes: their descriptor
    and workspace size when the caller has them).  The outputs are views of
    ONE zeroed float64 buffer ("_flat": results | scales | scale_errs |
    channel_snrs | covariance), which a caller may download in one copy."""
    nsub = c1 - c0
    nchan = per_sub["data"].shape[1]
    R = _lib.RESULT_DOUBLES
    sizes = (nsub * R, nsub * nchan, nsub * nchan, nsub * nchan, nsub * 25)
    flat = torch.zeros(sum(sizes), dtype=torch.float64, device=dev)
    views, o = [], 0
    for n in sizes:
        views.append(flat[o:o + n])
        o += n
    results = views[0].view(nsub, R)
    scales, scale_errs, channel_snrs = (v.view(nsub, nchan)
                                        for v in views[1:4])
    cov = views[4].view(nsub, 5, 5)
    if d is None:
        d = _desc(per_sub, c0, c1, n_x, cfg)
    if nbytes is None:
        nbytes = _desc_workspace_bytes(lib, d)
    d.results, d.scales, d.scale_errs = _p(results), _p(scales), \
        _p(scale_errs)
    d.channel_snrs, d.covariance = _p(channel_snrs), _p(cov)
    if workspace is None or workspace.numel() < nbytes or \
            workspace.device != dev:
        workspace = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d.workspace, d.workspace_bytes = _p(workspace), workspace.numel()
    ctx = _lib.context(dev.index)
    with span("fit.lib"):
        rc = lib.ppf_fit_batch(ctx, ctypes.byref(d), _stream(dev))
    _lib.check(rc, ctx)
    # keep inputs alive until the stream has consumed them
    keep = (cfg["model"],) + tuple(v for v in per_sub.values()
                                   if v is not None)
    return dict(results=results, scales=scales, scale_errs=scale_errs,
                channel_snrs=channel_snrs, covariance=cov,
                workspace=workspace, _keep=keep, _flat=flat)


def rotate_rows(rows, phases, dev=None, ref_len=False):
    """irfft(rfft(row) * exp(2 pi i k phase)) for each row of rows [..., nbin]
    (float64 output, same leading shape).  ref_len: the reference's public
    rotate routines' length-less irfft (ppf_rotate_batch_ref): nbin - 1
    samples per row at odd nbin; otherwise (internal callers) nbin."""
    dev = device(dev)
    r = to_dev(rows, dev, _data_dtype(rows)) if isinstance(rows, torch.Tensor) \
        else host_to_dev(rows, dev, _data_dtype(rows))
    shape = r.shape
    nbin = shape[-1]
    r2 = r.reshape(-1, nbin).contiguous()
    ph = to_dev(phases, dev, torch.float64).reshape(-1).contiguous()
    if ph.numel() != r2.shape[0]:
        raise ValueError("need one phase per row")
    nout = nbin - 1 if (ref_len and nbin % 2) else nbin
    out = torch.empty((r2.shape[0], nout), dtype=torch.float64, device=dev)
    ctx = _lib.context(dev.index)
    lib = _lib.load()
    if not _noise_batch_len_ok(nbin):
        # past the LDS transforms (even > 8192, odd > 4095; the same rule as
        # ppf_noise_batch): Bluestein transforms both ways (ppf_rotate_long)
        nb = lib.ppf_rotate_long_workspace_bytes(r2.shape[0], nbin,
                                                 int(bool(ref_len)))
        if nb == 0:
            raise NotImplementedError(
                "rotation of %d-sample rows: past the 2^23-point transform"
                % nbin)
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        rc = lib.ppf_rotate_long(
            ctx, r2.shape[0], nbin,
            _lib.PPF_F32 if r2.dtype == torch.float32 else _lib.PPF_F64,
            _p(r2), _p(ph), _p(out), int(bool(ref_len)), _p(ws), nb,
            _stream(dev))
        _lib.check(rc, ctx)
        return out.reshape(tuple(shape[:-1]) + (nout,))
    fn = lib.ppf_rotate_batch_ref if ref_len else lib.ppf_rotate_batch
    rc = fn(ctx, r2.shape[0], nbin,
            _lib.PPF_F32 if r2.dtype == torch.float32 else _lib.PPF_F64,
            _p(r2), _p(ph), _p(out), _stream(dev))
    _lib.check(rc, ctx)
    return out.reshape(tuple(shape[:-1]) + (nout,))


def align_accum(data, phases, weights, out, wsum, dev=None):
    """ppalign accumulation on the device (ppf_align_accum):
    out[n] += sum_s w[s,n] rotate(data[s,n], phases[s,n]); wsum[n] += sum_s
    w[s,n].  data [nsub, nchan, nbin]; out [nchan, nbin] and wsum [nchan] are
    float64 device tensors updated in place."""
    dev = device(dev)
    d = to_dev(data, dev, _data_dtype(data))
    if d.dim() != 3:
        raise ValueError("data must be [nsub, nchan, nbin]")
    nsub, nchan, nbin = d.shape
    ph = to_dev(phases, dev, torch.float64).reshape(nsub, nchan).contiguous()
    w = to_dev(weights, dev, torch.float64).reshape(nsub, nchan).contiguous()
    if out.shape != (nchan, nbin) or out.dtype != torch.float64 or \
            wsum.shape != (nchan,) or wsum.dtype != torch.float64:
        raise ValueError("out must be float64 [nchan, nbin], wsum [nchan]")
    lib = _lib.load()
    if not _noise_batch_len_ok(nbin):
        # rows past the LDS transforms: the rotations on the long transforms
        # (ppf_rotate_long), the weighted sum over sub-ints on the stream;
        # rows of weight 0 contribute nothing whatever they hold
        rot = rotate_rows(d, ph, dev).reshape(nsub, nchan, nbin)
        wr = w.unsqueeze(-1)
        out += torch.where(wr != 0.0, wr * rot, 0.0).sum(dim=0)
        wsum += w.sum(dim=0)
        return out, wsum
    nbytes = lib.ppf_align_workspace_bytes(nsub, nchan, nbin)
    ws = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=dev)
    ctx = _lib.context(dev.index)
    rc = lib.ppf_align_accum(
        ctx, nsub, nchan, nbin,
        _lib.PPF_F32 if d.dtype == torch.float32 else _lib.PPF_F64,
        _p(d), _p(ph), _p(w), _p(out), _p(wsum), _p(ws), int(nbytes),
        _stream(dev))
    _lib.check(rc, ctx)
    return out, wsum


def align_phases(results, freqs, P, mask, scales, errs, dev=None):
    """ppalign's per-row rotation phases and weights from fit results
    (ppf_align_phases, ppalign.py:222-247): device tensors results [nsub,
    32], freqs / scales / errs [nsub, nchan] float64, P [nsub], mask [nsub,
    nchan] uint8 (or None) -> (phases, weights) [nsub, nchan] float64."""
    dev = device(dev)
    nsub, nchan = freqs.shape
    for t in (results, freqs, P, scales, errs):
        if t.dtype != torch.float64 or not t.is_contiguous():
            raise ValueError("align_phases takes contiguous float64 tensors")
    ph = torch.empty((nsub, nchan), dtype=torch.float64, device=dev)
    wt = torch.empty((nsub, nchan), dtype=torch.float64, device=dev)
    ctx = _lib.context(dev.index)
    rc = _lib.load().ppf_align_phases(
        ctx, nsub, nchan, _p(results), _p(freqs), _p(P),
        None if mask is None else _p(mask), _p(scales), _p(errs), _p(ph),
        _p(wt), _stream(dev))
    _lib.check(rc, ctx)
    return ph, wt


def resid_chi2_rows(rows, phases, model_rows, model_index, scales, errs, dof,
                    dev=None):
    """Per row: sum_t (rotate(row, phase) - scale * model_rows[index])^2 /
    err^2 / dof (ppf_resid_chi2_batch) -> float64 [nrows]."""
    dev = device(dev)
    r = to_dev(rows, dev, _data_dtype(rows))
    nbin = r.shape[-1]
    r2 = r.reshape(-1, nbin).contiguous()
    n = r2.shape[0]
    ph = to_dev(phases, dev, torch.float64).reshape(-1).contiguous()
    m = to_dev(model_rows, dev, torch.float64).reshape(-1, nbin).contiguous()
    mi = to_dev(model_index, dev, torch.int32).reshape(-1).contiguous()
    sc = to_dev(scales, dev, torch.float64).reshape(-1).contiguous()
    er = to_dev(errs, dev, torch.float64).reshape(-1).contiguous()
    if not (ph.numel() == mi.numel() == sc.numel() == er.numel() == n):
        raise ValueError("need one phase / model index / scale / err per row")
    if n and (int(mi.min()) < 0 or int(mi.max()) >= m.shape[0]):
        raise ValueError("model index out of range")
    if not _noise_batch_len_ok(nbin):
        # rows past the LDS transforms (round 6): the rotation on the long
        # transforms (ppf_rotate_long, full nbin as k_resid_chi2's), the
        # residual sum of squares on the stream
        rot = rotate_rows(r2, ph, dev)
        res = (rot - sc.unsqueeze(-1) * m[mi.long()]) / er.unsqueeze(-1)
        return (res * res).sum(dim=-1) / float(dof)
    out = torch.empty(n, dtype=torch.float64, device=dev)
    ctx = _lib.context(dev.index)
    rc = _lib.load().ppf_resid_chi2_batch(
        ctx, n, nbin, _lib.PPF_F32 if r2.dtype == torch.float32 else
        _lib.PPF_F64, _p(r2), _p(ph), _p(m), _p(mi), _p(sc), _p(er),
        float(dof), _p(out), _stream(dev))
    _lib.check(rc, ctx)
    return out


def pinned_host_array(shape, dtype=np.float32):
    """A NumPy array in page-locked host memory (a torch pinned buffer; the
    array keeps it alive).  An archive loaded into one is uploaded by
    GetTOAs' stager straight from it, without the copy into its own pinned
    buffers."""
    t = torch.empty(tuple(shape), dtype=torch.from_numpy(
        np.zeros(0, dtype=dtype)).dtype, pin_memory=True)
    return t.numpy()


def _noise_batch_len_ok(nbin):
    """Row lengths ppf_noise_batch's LDS transforms take (nbin_supported)."""
    return 32 <= nbin <= 8192 and (nbin % 2 == 0 or nbin <= 4095)


def noise_rows(rows, frac=4, dev=None):
    """get_noise_PS per row of rows [..., nbin] -> [...] float64 (rows past
    the LDS transforms: ppf_noise_long)."""
    dev = device(dev)
    r = to_dev(rows, dev, _data_dtype(rows))
    shape = r.shape
    r2 = r.reshape(-1, shape[-1]).contiguous()
    if not _noise_batch_len_ok(shape[-1]):
        return noise_rows_long(r2, frac, dev).reshape(shape[:-1])
    out = torch.empty(r2.shape[0], dtype=torch.float64, device=dev)
    ctx = _lib.context(dev.index)
    rc = _lib.load().ppf_noise_batch(
        ctx, r2.shape[0], shape[-1],
        _lib.PPF_F32 if r2.dtype == torch.float32 else _lib.PPF_F64,
        _p(r2), int(frac), _p(out), _stream(dev))
    _lib.check(rc, ctx)
    return out.reshape(shape[:-1])


# largest prime factor of the transform length the LDS path takes for
# get_noise_PS of a single flattened row: the generic-radix stage costs
# O(N R) per row (R the prime), so a length like 8186 = 2 x 4093 would be a
# 4093-point direct DFT inside one workgroup; ppf_noise_long's Bluestein
# transform is faster
NOISE_MAX_PRIME = 61


def _max_prime_factor(n):
    p, m, f = 2, n, 1
    while p * p <= m:
        while m % p == 0:
            f, m = p, m // p
        p += 1
    return max(f, m) if m > 1 else f


def noise_len_supported(n):
    """Row lengths get_noise_PS(chans=False) sends to ppf_noise_batch (its LDS
    FFT): even 32..8192 or odd 33..4095 (every length ppf_noise_batch
    accepts) whose transform length -- n / 2 complex points at even n, n at
    odd n -- has no prime factor above NOISE_MAX_PRIME; the rest go to
    ppf_noise_long (noise_long)."""
    if not 32 <= n <= (8192 if n % 2 == 0 else 4095):
        return False
    return _max_prime_factor(n // 2 if n % 2 == 0 else n) <= NOISE_MAX_PRIME


def noise_rows_long(rows, frac=4, dev=None):
    """get_noise_PS of rows [nrows, nbin] of any length (pplib.py:2312-2338)
    on ppf_noise_long: a four-step rFFT of block LDS transforms, or
    Bluestein's chirp z-transform on one, up to 2^24 complex points ->
    [nrows] float64 on the device."""
    dev = device(dev)
    r = to_dev(rows, dev, _data_dtype(rows))
    r2 = r.reshape(-1, r.shape[-1]).contiguous()
    nrows, nbin = r2.shape
    lib = _lib.load()
    nb = lib.ppf_noise_long_workspace_bytes(nrows, nbin)
    if nb == 0:
        raise NotImplementedError(
            "get_noise_PS of %d-sample rows: past the 2^24-point transform"
            % nbin)
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    out = torch.empty(nrows, dtype=torch.float64, device=dev)
    ctx = _lib.context(dev.index)
    rc = lib.ppf_noise_long(
        ctx, nrows, nbin,
        _lib.PPF_F32 if r2.dtype == torch.float32 else _lib.PPF_F64,
        _p(r2), int(frac), _p(out), _p(ws), nb, _stream(dev))
    _lib.check(rc, ctx)
    return out


def noise_long(row, frac=4, dev=None):
    """get_noise_PS of ONE row of any length (pplib.py:2334-2338: the
    flattened portrait of get_noise(chans=False)): the mean power of the top
    1/frac of the rFFT, float64 (ppf_noise_long)."""
    x = to_dev(row, device(dev), None if isinstance(row, torch.Tensor)
               else torch.float64)
    return float(noise_rows_long(x.reshape(1, -1), frac, dev).cpu()[0])


def unpack_psrfits(raw, elem, npol, nchan, nbin, scl, offs, wts=None,
                   pol_mode=0, rm_baseline=True, dev=None):
    """ppf_unpack_psrfits_batch: raw DATA bytes [nsub, >= npol nchan nbin
    esize] (device uint8 tensor, one row per sub-int, as stored in the
    file) -> dict(rows float32 [nsub, nchan, nbin], stats float64
    [nsub, nchan, 3] (off-pulse mean, sigma, S/N), total float64
    [nsub, nbin], wstart int32 [nsub]), all on the device."""
    dev = device(dev)
    nsub = raw.shape[0]
    f32 = torch.float32
    scl_t = to_dev(scl, dev, f32).reshape(nsub, npol * nchan).contiguous()
    offs_t = to_dev(offs, dev, f32).reshape(nsub, npol * nchan).contiguous()
    wts_t = None if wts is None else \
        to_dev(wts, dev, f32).reshape(nsub, nchan).contiguous()
    rows = torch.empty((nsub, nchan, nbin), dtype=f32, device=dev)
    stats = torch.empty((nsub, nchan, 3), dtype=torch.float64, device=dev)
    total = torch.empty((nsub, nbin), dtype=torch.float64, device=dev)
    wstart = torch.empty(nsub, dtype=torch.int32, device=dev)
    lib = _lib.load()
    wsb = int(lib.ppf_unpack_workspace_bytes(nsub, nchan, nbin))
    ws = torch.empty(max(wsb, 8), dtype=torch.uint8, device=dev)
    ctx = _lib.context(dev.index)
    rc = lib.ppf_unpack_psrfits_batch(
        ctx, nsub, npol, nchan, nbin, int(elem), _p(raw), int(raw.stride(0)),
        _p(scl_t), _p(offs_t), None if wts_t is None else _p(wts_t),
        int(pol_mode), int(bool(rm_baseline)), _p(rows), _p(stats), _p(total),
        _p(wstart), _p(ws), wsb, _stream(dev))
    _lib.check(rc, ctx)
    return dict(rows=rows, stats=stats, total=total, wstart=wstart,
                _keep=(scl_t, offs_t, wts_t, ws, raw))


def scales_batch(D, M, params, P, freqs, nus, log10_tau, errs_FT=None,
                 model_index=None, dev=None):
    """get_scales_full (pptoaslib.py:953-971) per sub-int: D [nsub, nchan,
    nharm] complex data spectra, M [nmodel, nchan, nharm] complex model
    spectra (or [nchan, nharm]), params [nsub, 5], P [nsub], freqs
    [nsub, nchan], nus [nsub, 3]; returns a_n [nsub, nchan] float64."""
    dev = device(dev)
    c128 = torch.complex128
    D_t = to_dev(D, dev, c128)
    if D_t.dim() == 2:
        D_t = D_t.unsqueeze(0)
    nsub, nchan, nharm = D_t.shape
    M_t = to_dev(M, dev, c128)
    if M_t.dim() == 2:
        M_t = M_t.unsqueeze(0)
    if M_t.shape[1:] != (nchan, nharm):
        raise ValueError("model spectra %s != [*, %d, %d]" %
                         (tuple(M_t.shape), nchan, nharm))
    f64 = torch.float64
    pr = to_dev(params, dev, f64).reshape(nsub, 5).contiguous()
    P_t = to_dev(np.broadcast_to(np.asarray(P, dtype=float), (nsub,)).copy()
                 if not isinstance(P, torch.Tensor) else P, dev, f64)
    fr = to_dev(freqs, dev, f64).reshape(-1)
    if fr.numel() == nchan:
        fr = fr.repeat(nsub)
    fr = fr.reshape(nsub, nchan).contiguous()
    nu = to_dev(nus, dev, f64).reshape(-1)
    if nu.numel() == 3:
        nu = nu.repeat(nsub)
    nu = nu.reshape(nsub, 3).contiguous()
    e_t = None if errs_FT is None else \
        to_dev(errs_FT, dev, f64).reshape(-1)
    if e_t is not None and e_t.numel() == nchan:
        e_t = e_t.repeat(nsub)
    mi = None if model_index is None else \
        to_dev(model_index, dev, torch.int32).reshape(nsub).contiguous()
    out = torch.empty((nsub, nchan), dtype=f64, device=dev)
    ctx = _lib.context(dev.index)
    rc = _lib.load().ppf_scales_batch(
        ctx, nsub, nchan, nharm, _p(D_t), _p(M_t), _p(mi), _p(e_t), _p(pr),
        _p(P_t), _p(fr), _p(nu), int(bool(log10_tau)), _p(out), _stream(dev))
    _lib.check(rc, ctx)
    return out


def phase_shift_batch(data, model, noise=None, Ns=100, bounds=(-0.5, 0.5),
                      model_index=None, dev=None):
    """Batched pplib.fit_phase_shift: data [nprof, nbin], model
    [nmodel, nbin] -> [nprof, 8] (phase, phase_err, scale, scale_err, snr,
    red_chi2, nfev, status)."""
    dev = device(dev)
    d = to_dev(data, dev, _data_dtype(data))
    if d.dim() == 1:
        d = d.unsqueeze(0)
    m = to_dev(model, dev, torch.float64)
    if m.dim() == 1:
        m = m.unsqueeze(0)
    nz = None if noise is None else \
        to_dev(noise, dev, torch.float64).reshape(-1).contiguous()
    mi = None if model_index is None else \
        to_dev(model_index, dev, torch.int32).reshape(-1).contiguous()
    out = torch.zeros((d.shape[0], 8), dtype=torch.float64, device=dev)
    ctx = _lib.context(dev.index)
    rc = _lib.load().ppf_phase_shift_batch(
        ctx, d.shape[0], d.shape[1],
        _lib.PPF_F32 if d.dtype == torch.float32 else _lib.PPF_F64,
        _p(d), _p(m), _p(mi), _p(nz), int(Ns), float(bounds[0]),
        float(bounds[1]), _p(out), _stream(dev))
    _lib.check(rc, ctx)
    return out


def gauss_portraits(model_code, params, scattering_index, freqs, nu_ref, nbin,
                    dev=None):
    """Gaussian-component model portraits (pplib.gen_gaussian_portrait,
    pplib.py:886-963) on the device: params [nport, 2 + 6 ngauss] (DC, tau
    [bin], per component loc, m_loc, wid, m_wid, amp, m_amp),
    scattering_index [nport], freqs [nport, nchan], nu_ref [nport] ->
    float64 [nport, nchan, nbin] (odd nbin with tau != 0: nbin - 1 bins, as
    the reference's length-less irfft gives, then a zero column)."""
    code = str(model_code)
    if len(code) != 3 or any(c not in "01" for c in code):
        raise KeyError(code)     # evolve_parameter's dictionary lookup
    dev = device(dev)
    prm = to_dev(params, dev, torch.float64)
    if prm.dim() == 1:
        prm = prm.unsqueeze(0)
    nport, npar = prm.shape
    if npar < 2 or (npar - 2) % 6:
        raise ValueError("params must hold 2 + 6*ngauss values per portrait")
    f = to_dev(freqs, dev, torch.float64).reshape(nport, -1).contiguous()
    nchan = f.shape[1]
    si = to_dev(np.broadcast_to(np.asarray(scattering_index, dtype=float),
                                (nport,)), dev, torch.float64).contiguous()
    nr = to_dev(np.broadcast_to(np.asarray(nu_ref, dtype=float), (nport,)),
                dev, torch.float64).contiguous()
    out = torch.empty((nport, nchan, int(nbin)), dtype=torch.float64,
                      device=dev)
    ctx = _lib.context(dev.index)
    rc = _lib.load().ppf_gauss_portrait_batch(
        ctx, nport, nchan, int(nbin), (npar - 2) // 6, code.encode(),
        _p(prm), _p(si), _p(f), _p(nr), _p(out), _stream(dev))
    _lib.check(rc, ctx)
    return out


def spline_portraits(mean_prof, eigvec, tck, freqs, nbin=None, dev=None):
    """PCA + B-spline model portraits (pplib.gen_spline_portrait,
    pplib.py:966-990) on the device (ppf_spline_portrait_batch): mean_prof
    [nbin_model], eigvec [nbin_model, ncomp], tck = (knots, [coefs per
    component], degree) as si.splprep returns it, freqs [nport, nchan] (or
    [nchan]) -> float64 [nport, nchan, nbin]."""
    dev = device(dev)
    mean_prof = np.asarray(mean_prof, dtype=np.float64)
    eigvec = np.asarray(eigvec, dtype=np.float64)
    nbin0 = len(mean_prof)
    nbin = nbin0 if nbin is None else int(nbin)
    ncomp = eigvec.shape[1] if eigvec.ndim == 2 else 0
    f = np.atleast_2d(np.asarray(freqs, dtype=np.float64))
    nport, nchan = f.shape
    if ncomp:
        t = np.asarray(tck[0], dtype=np.float64)
        cs = [np.asarray(c, dtype=np.float64) for c in tck[1]]
        if len(cs) != ncomp:
            raise ValueError("tck has %d coefficient arrays, eigvec %d "
                             "columns" % (len(cs), ncomp))
        coefs = np.zeros((ncomp, len(t)))
        for i, c in enumerate(cs):
            coefs[i, :len(c)] = c
        degree, nknots = int(tck[2]), len(t)
    else:
        t, coefs, degree, nknots = np.zeros(1), np.zeros((1, 1)), 0, 1
    ev = eigvec if ncomp else np.zeros((nbin0, 1))
    mp_t = to_dev(mean_prof, dev, torch.float64)
    ev_t = to_dev(np.ascontiguousarray(ev), dev, torch.float64)
    t_t = to_dev(t, dev, torch.float64)
    c_t = to_dev(coefs, dev, torch.float64)
    f_t = to_dev(f, dev, torch.float64)
    out = torch.empty((nport, nchan, nbin), dtype=torch.float64, device=dev)
    ctx = _lib.context(dev.index)
    rc = _lib.load().ppf_spline_portrait_batch(
        ctx, nport, nchan, nbin0, nbin, ncomp, nknots, degree, _p(mp_t),
        _p(ev_t), _p(t_t), _p(c_t), _p(f_t), _p(out), _stream(dev))
    _lib.check(rc, ctx)
    return out


def synth(model, freqs, phi, DM, P, nu_ref, noise, seed, out_dtype=torch.float32,
          dev=None, first=0):
    """Synthetic sub-integrations [nsub, nchan, nbin] on the device."""
    dev = device(dev)
    m = to_dev(model, dev, torch.float64)
    nchan, nbin = m.shape
    f = to_dev(freqs, dev, torch.float64).reshape(-1).contiguous()
    ph = to_dev(phi, dev, torch.float64).reshape(-1).contiguous()
    dm = to_dev(DM, dev, torch.float64).reshape(-1).contiguous()
    Pt = to_dev(P, dev, torch.float64).reshape(-1).contiguous()
    nsub = ph.numel()
    out = torch.empty((nsub, nchan, nbin), dtype=out_dtype, device=dev)
    ctx = _lib.context(dev.index)
    rc = _lib.load().ppf_synth_batch(
        ctx, nsub, nchan, nbin, _p(m), _p(f), _p(ph), _p(dm), _p(Pt),
        float(nu_ref), float(noise), ctypes.c_uint64(int(seed)), int(first),
        _lib.PPF_F32 if out_dtype == torch.float32 else _lib.PPF_F64,
        _p(out), _stream(dev))
    _lib.check(rc, ctx)
    return out


def results_numpy(res):
    """Device fit_batch output -> dict of numpy arrays (synchronises)."""
    out = {k: v.detach().cpu().numpy() for k, v in res.items()
           if isinstance(v, torch.Tensor) and k != "workspace"}
    return out

#!/usr/bin/env python
"""Headline benchmark: subint portrait fits/sec (phase+DM, 512ch x 2048bin).

Workload (BASELINE.json configs[1]): synthetic 512-channel x 2048-bin
sub-integrations, N_sub per GPU (default 10,000), the full GetTOAs hot path
per sub-integration on the device: power-spectrum noise, cross spectrum,
initial phase from the dedispersed mean profile (brute grid + Nelder-Mead),
the trust-region wideband fit (phi, DM), zero-covariance frequency, output
transform, covariance, scales and S/N.  Inputs are resident in HBM (float32
amplitudes, generated on the device) before the timed region; one "step" =
one pass of the hot path over the whole batch, plus the RCCL all-gather of
the result records when N > 1 (weak scaling: N_sub per GPU is fixed).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

With --gpus N > 1 and no launcher (WORLD_SIZE unset), bench.py starts its N
ranks itself (one child process per GPU, dist.launch_local) and forwards
rank 0's JSON line; under torchrun / torch.distributed.run each process is
one rank.

Rank 0 prints ONE JSON line.  It carries `roofline` for the dominant kernel
(algorithmic bytes from HIP events around each kernel on the launch stream)
and `cpu_baseline` (the NumPy/SciPy oracle on a bounded sample, 1 core).
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = ("subint portrait fits/sec (phase+DM, 512ch×2048bin) at "
          "1/2/4/8 MI355X")
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP64_PEAK_TF = 78.6            # MI355X spec: FP64 vector = FP64 matrix = 78.6 TFLOPS (half the 157.3 FP32 rate, MI355X_MICROARCH.md)


MOMX = {"auto": None, "x": True, "fused": False}
# who started the ranks: "bench-self" (bench.py --gpus N started its own),
# "env" (WORLD_SIZE came from the environment: torchrun / torch.distributed.run),
# or "none" (N = 1)
LAUNCHER = os.environ.get("PPF_LAUNCHER") or (
    "env" if "WORLD_SIZE" in os.environ else "none")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nsub", type=int, default=10000,
                    help="sub-integrations per GPU")
    ap.add_argument("--nchan", type=int, default=512)
    ap.add_argument("--nbin", type=int, default=2048)
    ap.add_argument("--chunk", type=int, default=None,
                    help="sub-integrations per ppf_fit_batch call (default: "
                    "all of a GPU's sub-ints; scattering fits: at most ~150 "
                    "GB of cross spectrum per call)")
    ap.add_argument("--fit", default="phase+DM",
                    choices=["phase+DM", "full", "scat", "align",
                             "gettoas", "single"],
                    help="phase+DM: configs[1] (the metric); full: configs[2] "
                    "fit (phi, DM, GM, tau, alpha) on data with injected "
                    "scattering; scat: configs[4] fit (phi, DM, tau, alpha), "
                    "CHIME-like band; align: configs[3] ppalign iteration "
                    "(--nsub archives, default shape 256 x 1024); gettoas: "
                    "end-to-end GetTOAs.get_TOAs over host archives of "
                    "--arch-nsub sub-ints (default --nsub 2048); single: "
                    "single-call latency of fit_portrait_full / fit_portrait /"
                    " rotate_data at 64x512 and 512x2048")
    ap.add_argument("--arch-nsub", type=int, default=64,
                    help="sub-ints per archive for --fit gettoas")
    ap.add_argument("--pinned", action="store_true",
                    help="--fit gettoas: archives held in page-locked host "
                    "memory (uploaded without the staging copy)")
    ap.add_argument("--psrfits", action="store_true",
                    help="--fit gettoas: archives written as fold-mode "
                    "PSRFITS files (16-bit DATA + DAT_SCL/DAT_OFFS, one "
                    "polarisation) and read through the PSRCHIVE-free fast "
                    "path (raw bytes to the device, unpacked there)")
    ap.add_argument("--timeline", default=None,
                    help="--fit gettoas: write the host timeline of the "
                    "last timed step (pulseportraiture_amd.timeline spans, "
                    "per stage and thread) to this JSON file")
    ap.add_argument("--zap-frac", type=float, default=0.0,
                    help="fraction of channels masked (zapped) in every "
                    "sub-int, as GetTOAs passes its ok_ichans (default 0)")
    ap.add_argument("--passes", type=int, default=None,
                    help="fits of every resident sub-int per step (default "
                    "phase+DM: 24, so the driver's 20 timed steps span >10 s "
                    "of GPU work; other fits: 1)")
    ap.add_argument("--no-hcut", action="store_true",
                    help="sum every harmonic (PPF_OPT_NO_HCUT: no per-channel "
                    "cutoff of harmonics below 1e-28 of the template's peak "
                    "power)")
    ap.add_argument("--mom-x", default="auto", choices=["auto", "x", "fused"],
                    help="where phase/DM fits take their Taylor moments: "
                    "the library's choice (auto: from the stored cross "
                    "spectrum at nbin 2048 with the guess fused into the "
                    "spectrum pass), always from X (k_xspec_w + k_moments, "
                    "PPF_OPT_MOM_X) or always from the fused k_xmom_g pass "
                    "(PPF_OPT_FUSED_MOM)")
    ap.add_argument("--solver", default="newton", choices=["newton", "scipy"],
                    help="minimiser of the scattering fits (--fit full/scat): "
                    "the Newton trust region (default) or scipy trust-ncg's "
                    "own path (PPF_OPT_SCIPY_TR)")
    ap.add_argument("--cpu-sample", type=int, default=48,
                    help="sub-integrations for the CPU baseline (0: skip)")
    ap.add_argument("--cpu-workers", type=int, default=16,
                    help="processes for the all-core CPU aggregate (the GPU "
                    "box's CPU share is 16)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend at N > 1 (nccl = RCCL; gloo "
                    "only to rehearse several ranks on one GPU)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles",
                                                  "pmc_summary.json"))
    return ap.parse_args()


def _noop(_):
    return 0


def _warm_worker():
    import oracle.ppfit_oracle  # noqa: F401  (import NumPy/SciPy up front)
    import scipy.optimize  # noqa: F401


def _oracle_toas(O, data, model, freqs, P, DM0, flags):
    """The oracle's get_TOAs loop over rows [n, nchan, nbin] (the bench's
    guesses: DM_stored = DM0; scattering fits start from log10 tau = log10
    (1 / nbin), alpha = -4, pptoas.py:467-492)."""
    n, nchan = data.shape[:2]
    return O.get_toas_archive(data, model, np.tile(freqs, (n, 1)),
                              np.ones((n, nchan)), np.ones((n, nchan)), P, DM0,
                              np.ones(n), fit_flags=tuple(flags),
                              tau_guess=0.0, alpha_guess=-4.0, log10_tau=True)


def _oracle_chunk(args):
    """One worker of the all-core CPU aggregate (a child process)."""
    data, model, freqs, P, DM0, flags = args
    import oracle.ppfit_oracle as O
    from threadpoolctl import threadpool_limits
    with threadpool_limits(1):
        t0 = time.perf_counter()
        out = _oracle_toas(O, data, model, freqs, P, DM0, flags)
        return time.perf_counter() - t0, {k: out[k] for k in _PARITY_KEYS}


# the oracle outputs parity_vs_oracle reads
_PARITY_KEYS = ("phis", "phi_errs", "DMs", "DM_errs", "nu_refs", "param_errs",
                "red_chi2s", "GMs", "taus", "alphas")


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


def cpu_baseline(batch, nsample, nchan, nbin, workers, mode="phase+DM",
                 flags=(1, 1, 0, 0, 0), per_worker=4):
    """Oracle (NumPy/SciPy restatement of the reference get_TOAs inner loop:
    noise, FFTFIT guess, trust-ncg fit, post-fit) on `nsample`
    sub-integrations of the same workload: one core, then `workers` processes
    (one core each) on 2 x workers more sub-ints for the all-core aggregate.
    Returns (baseline dict, the one-core oracle outputs for the parity
    check)."""
    import oracle.ppfit_oracle as O
    from threadpoolctl import threadpool_limits
    data = batch["data"][:nsample].double().cpu().numpy()
    freqs = np.tile(batch["freqs"], (nsample, 1))
    with threadpool_limits(1):
        t0 = time.perf_counter()
        ref = _oracle_toas(O, data, batch["model"], batch["freqs"],
                           batch["P"][:nsample], O_DM0(), flags)
        dt = time.perf_counter() - t0
    value = nsample / dt
    out = dict(value=value, unit="subint-fits/s", cores=1, kind="port",
               sample="%d sub-integrations of %dch x %dbin, oracle get_TOAs "
                      "loop (noise, FFTFIT guess, trust-ncg fit of %s, "
                      "post-fit), %.1f s" % (nsample, nchan, nbin, mode, dt),
               cpu_model=_cpu_model(), nproc=os.cpu_count())
    # reference-equivalent: the reference's loop is slower than the oracle by
    # a ratio measured in the build container on identical inputs
    # (tools/cpu_ratio.py -> profiles/cpu_ratio.json)
    rpath = os.path.join(ROOT, "profiles", "cpu_ratio.json")
    if os.path.exists(rpath):
        r = json.load(open(rpath))
        if mode == "phase+DM":
            ratio = r.get("reference_over_oracle_time")
        else:
            ratio = r.get("scattering_fits", {}).get(mode, {}).get(
                "reference_over_oracle_time")
        if ratio:
            out["reference_equiv_value"] = value / float(ratio)
            out["reference_over_oracle_time"] = round(float(ratio), 3)
    if workers > 1:
        import multiprocessing as mp
        n_all = min(per_worker * workers, batch["data"].shape[0])
        d_all = batch["data"][:n_all].double().cpu().numpy()
        jobs = [(d_all[i::workers], batch["model"], batch["freqs"],
                 batch["P"][:n_all][i::workers], O_DM0(), tuple(flags))
                for i in range(workers)]
        ctx = mp.get_context("spawn")
        with ctx.Pool(workers, initializer=_warm_worker) as pool:
            pool.map(_noop,
                     range(workers), chunksize=1)   # every worker started
            t0 = time.perf_counter()
            res = pool.map(_oracle_chunk, jobs, chunksize=1)
            wall = time.perf_counter() - t0
        out["all_core"] = dict(value=n_all / wall, workers=workers,
                               cores=workers,
                               sample="%d sub-ints, %d processes x 1 thread "
                                      "(the box's CPU share), %.1f s wall" %
                                      (n_all, workers, wall))
        # the workers' fits (worker i fitted sub-ints i, i + workers, ...)
        # in global order: the parity sample of the all-core run
        allref = {}
        for k in _PARITY_KEYS:
            first = np.asarray(res[0][1][k])
            a = np.zeros((n_all,) + first.shape[1:])
            for i in range(workers):
                a[i::workers] = np.asarray(res[i][1][k])
            allref[k] = a
        ref = dict(ref, all_core=allref, n_all=n_all)
    return out, ref


def parity_vs_oracle(R, o, P, flags=(1, 1, 0, 0, 0)):
    """The device fits of the cpu_baseline sub-ints against the oracle's
    fits of the same sub-ints: worst parameter deviation in units of the
    oracle's uncertainty (phase compared at the oracle's nu_DM; GM, log10
    tau and alpha when fitted) and worst relative chi2_red difference (bar:
    0.01 sigma, 1e-8)."""
    from pulseportraiture_amd import _lib
    I = _lib.RESULT_INDEX
    D = 0.000241 ** -1
    dev, rel = 0.0, 0.0
    for i in range(len(R)):
        phi, DM = R[i, I["params"]][:2]
        nu_d = R[i, I["nu_out"]][0]
        nu_o = o["nu_refs"][i][0]
        phi_o = phi + D * DM / P[i] * (nu_o ** -2 - nu_d ** -2)
        dphi = (phi_o - o["phis"][i] + 0.5) % 1.0 - 0.5
        dev = max(dev, abs(dphi) / o["phi_errs"][i],
                  abs(DM - o["DMs"][i]) / o["DM_errs"][i])
        for j, key in ((2, "GMs"), (3, "taus"), (4, "alphas")):
            if flags[j]:
                dev = max(dev, abs(R[i, I["params"]][j] - o[key][i]) /
                          o["param_errs"][i][j])
        rel = max(rel, abs(R[i, I["red_chi2"]] / o["red_chi2s"][i] - 1.0))
    return dict(n=int(len(R)), max_dev_sigma=float(dev),
                max_rchi2_rel=float(rel),
                ok=bool(dev < 0.01 and rel < 1e-8),
                against="oracle get_TOAs loop on the cpu_baseline sub-ints")


def O_DM0():
    from pulseportraiture_amd.synth import DM0
    return DM0



def _solver_fp64(fk, parts, nchan, nmom, evaluations, fpath):
    """The bench line's solver_fp64 object: per solver kernel (key, name,
    event-timed ms, units or None, launches) its f64 flops from the SQ
    passes (fp64_summary.json entry fk) over its time, against the fp64
    peak; k_tr_mom also its memory-side rate (it re-reads the moment set of
    every channel on every evaluation: nmom complex moments plus the channel
    scalars and the radius test's dphi / centre residual; the sets outgrow
    the L2s, re-reads of one sub-int's set within a launch may hit the MALL)."""
    items = {}
    tot_fl = tot_ms = 0.0
    for key, name, ms, units, nl in parts:
        k = fk.get(key)
        it = dict(name=name, total_ms=round(float(ms), 3), launches=int(nl))
        if k is not None and ms > 0:
            # units: sub-ints (or sub-int evaluations); k_tr_mom and
            # k_tr_step count per launch in the SQ pass's units, so their
            # units follow from the profiled run's ratio
            if units is None:
                units = k["units"] / max(k["dispatches"], 1) * nl
            fl = k["flops_per_unit"] * units
            tf = fl / (ms / 1e3) / 1e12
            it.update(flops_per_unit=round(k["flops_per_unit"]),
                      achieved_tflops=round(tf, 3),
                      frac=round(tf / FP64_PEAK_TF, 4),
                      valu_active_per_wave=k.get("valu_active_per_wave"))
            tot_fl += fl
            tot_ms += ms
        if key == "tr_mom" and ms > 0:
            bpe = nchan * (nmom * 16 + 40 + 32)
            mb = evaluations * bpe
            it["memory"] = dict(bytes_per_evaluation=bpe,
                                evaluations=round(evaluations),
                                achieved_gbs=round(mb / (ms / 1e3) / 1e9, 1),
                                hbm_frac=round(mb / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4))
        items[key] = it
    return dict(bound="fp64", peak=FP64_PEAK_TF, unit="TFLOP/s",
                achieved=round(tot_fl / max(tot_ms, 1e-9) / 1e9, 3) if tot_ms else None,
                frac=round(tot_fl / max(tot_ms, 1e-9) / 1e9 / FP64_PEAK_TF, 4) if tot_ms else None,
                kernels=items, source=os.path.relpath(fpath, ROOT))

def bench_align(args):
    """configs[3]: ppalign.align_archives iterations over --nsub tscrunched
    archives (256 ch x 1024 bin by default).  One step = one iteration: the
    batched guess + phase/DM fit of every archive against the current
    template, the weighted rotate-and-sum (ppf_align_accum), normalisation,
    (+ the all-reduce of the portrait at N > 1).  Sharded by archive."""
    import torch
    from types import SimpleNamespace
    from pulseportraiture_amd import dist, engine, ppalign, synth
    from pulseportraiture_amd.pplib import guess_fit_freq
    rank, world, local = dist.init(args.dist_backend)
    dev = torch.device("cuda", local)
    total = args.nsub * world
    first, count = dist.shard(total, rank, world)
    nchan, nbin = args.nchan, args.nbin
    b = synth.make_batch(count, nchan, nbin, first=first, dev=dev)
    noise = engine.noise_rows(b["data"]).cpu().numpy()     # get_noise_PS
    freqs = np.tile(b["freqs"], (count, 1))
    R = SimpleNamespace(
        n=count, data=b["data"][:, None], freqs=freqs,
        mask=np.ones((count, nchan), np.uint8), errs=noise,
        gw=np.ones((count, nchan)), P=b["P"],
        DM_guess=np.full(count, synth.DM0),
        nu_fit=np.full(count, guess_fit_freq(b["freqs"])),
        nchanx=np.full(count, nchan))
    # initial template (the reference notebook's
    # make_constant_portrait(profile=DataPortrait.prof)): archive 0's mean
    # profile, dedispersed at DM0 to the band centre, tiled
    D = 0.000241 ** -1
    ded = engine.rotate_rows(b["data"][0], D * synth.DM0 * (
        b["freqs"] ** -2 - 1500.0 ** -2) / b["P"][0])
    prof = ded.mean(dim=0).cpu().numpy()
    model0 = np.tile(prof, (nchan, 1))
    comm = dist.is_dist()
    from pulseportraiture_amd import _lib
    lib = _lib.load()
    lctx = _lib.context(dev.index)
    lib.ppf_set_profiling(lctx, 1)
    acc_ev = []                     # HIP events around ppf_align_accum

    def step(model_port, R=R, timed=True):
        out = torch.zeros((nchan, nbin), dtype=torch.float64, device=dev)
        wsum = torch.zeros(nchan, dtype=torch.float64, device=dev)
        ph, w = ppalign._fit_and_weights(R, model_port, True, nbin, dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), \
            torch.cuda.Event(enable_timing=True)
        e0.record()
        engine.align_accum(R.data[:, 0], ph, w, out, wsum, dev=dev)
        e1.record()
        if timed:
            acc_ev.append((e0, e1))
        ppalign.raise_pending(R)
        if comm:
            dist.allreduce_sum_(out, wsum)
        out /= torch.where(wsum > 0, wsum, torch.ones_like(wsum))[:, None]   # as ppalign
        return out                      # the next template stays in HBM

    m = model0
    for _ in range(args.warmup):
        m = step(m)
    torch.cuda.synchronize(dev)
    dist.barrier()
    m = model0 if args.warmup == 0 else m
    del acc_ev[:]
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m = step(m)
    torch.cuda.synchronize(dev)
    dist.barrier()
    dt = dist.max_over_ranks(time.perf_counter() - t0, dev)
    value = total * args.steps / dt
    # ---- per-kernel times of the timed region (HIP events on the stream) ---
    ncalls = args.steps                     # one ppf_fit_batch per iteration
    khist = np.zeros((ncalls, 2))
    kgot = lib.ppf_kernel_ms_history(lctx, ncalls, khist.ctypes.data)
    kern_ms = khist[:kgot].sum(axis=0)
    acc_ms = float(sum(a.elapsed_time(b) for a, b in acc_ev))
    nharm = nbin // 2 + 1
    nblkd = (nchan + 127) // 128
    # ALGORITHMIC bytes per archive: k_xmom_g reads the
    # f32 rows and the channel derivatives, writes 32 complex moments + 4
    # scalars + the centre residual per channel (+ the model spectra once per
    # launch); k_dsum_w reads the rows and writes the block guess profiles;
    # k_align reads the rows and the channel phases / weights (+ writes the
    # template and its weights once per launch)
    xmom_unit = nchan * nbin * 4 + nchan * 16 + nchan * (32 * 16 + 4 * 8 + 8)
    dsum_unit = nchan * nbin * 4 + nblkd * nbin * 8 + nblkd * 16
    acc_unit = nchan * nbin * 4 + nchan * 16
    L2N = (nbin // 4).bit_length()
    kern = {
        "xmom": dict(name="k_xmom_g<%d, 0, true, true>" % L2N, ms=kern_ms[0],
                     unit=xmom_unit, bytes=ncalls * (count * xmom_unit +
                                                     nchan * nharm * 16)),
        "dsum": dict(name="k_dsum_w" if (nbin & (nbin - 1)) == 0 else "k_dsum_wn",
                     ms=kern_ms[1], unit=dsum_unit,
                     bytes=ncalls * count * dsum_unit),
        "accum": dict(name="k_align", ms=acc_ms, unit=acc_unit,
                      bytes=ncalls * (count * acc_unit + nchan * nbin * 8 +
                                      nchan * 8)),
    }
    dom = max(kern, key=lambda k: kern[k]["ms"])
    dk = kern[dom]
    achieved = dk["bytes"] / (dk["ms"] / 1e3) / 1e9
    # HBM traffic per launch from the PMC passes of the same command
    # (profiles/pmc_reduce.py, mode "align")
    traffic = None
    if os.path.exists(args.pmc):
        pm = json.load(open(args.pmc)).get("modes", {}).get("align", {})
        same = ("%dch x %dbin" % (nchan, nbin)) in str(
            (pm.get("source") or {}).get("bench", ""))
        pk = pm.get("kernels", {}).get(dom) if same else None
        if pk:
            traffic = round(pk["hbm_bytes"] * count)
    roof = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS,
                unit="GB/s", frac=round(achieved / HBM_PEAK_GBS, 4),
                traffic=traffic, kernel=dk["name"],
                algorithmic_bytes_per_launch=dk["bytes"] / ncalls,
                algorithmic_bytes_per_unit=dk["unit"],
                avg_launch_ms=round(dk["ms"] / ncalls, 4), launches=ncalls,
                units_per_launch=count)
    kernels = {k: dict(name=v["name"], total_ms=round(float(v["ms"]), 3),
                       avg_launch_ms=round(float(v["ms"]) / ncalls, 4),
                       gbs=(None if not v["ms"] else
                            round(v["bytes"] / (v["ms"] / 1e3) / 1e9, 1)))
               for k, v in kern.items()}
    # solver kernels of the timed calls: [k_tr_mom ms, launches, k_tr_step
    # ms, launches, k_postfit ms, launches]
    shist = np.zeros((ncalls, 6))
    sgot = lib.ppf_solver_ms_history(lctx, ncalls, shist.ctypes.data)
    solv_ms = shist[:max(sgot, 0)].sum(axis=0)
    fitstats = {}
    lr = R.__dict__.get("_dev_inputs", {}).get("last_results")
    if lr is not None:
        from pulseportraiture_amd import _lib
        I = _lib.RESULT_INDEX
        lr = lr.cpu().numpy()
        fitstats = dict(mean_passes_per_fit=round(float(lr[:, I["npass"]].mean()), 3),
                        mean_evals_per_fit=round(float(lr[:, I["nfeval"]].mean()), 3),
                        passes_hist=np.bincount(lr[:, I["npass"]].astype(int)).tolist())
    # fp64 utilisation of the solver (as the fit modes' solver_fp64): the
    # moment sets come from the fused pass k_xmom_g (32 moments, priced in
    # the roofline above), every trust-region evaluation from k_tr_mom
    solver = None
    fpath = os.path.join(ROOT, "profiles", "fp64_summary.json")
    if os.path.exists(fpath) and fitstats:
        fm = json.load(open(fpath)).get("modes", {}).get("align", {})
        same = ("%dch x %dbin" % (nchan, nbin)) in str(
            (fm.get("source") or {}).get("bench", ""))
        if same:
            parts = [("tr_mom", "k_tr_mom", solv_ms[0], None, solv_ms[1]),
                     ("postfit", "k_postfit", solv_ms[4], ncalls * count, solv_ms[5])]
            solver = _solver_fp64(fm.get("kernels", {}), parts, nchan, 32,
                                  ncalls * count * fitstats["mean_evals_per_fit"], fpath)
    out = dict(metric="archive fits+aligns/sec (ppalign iteration, %dch×"
                      "%dbin) at 1/2/4/8 MI355X" % (nchan, nbin),
               value=round(value, 2), unit="archive-iterations/s",
               n_gpus=world, steps=args.steps, warmup=args.warmup,
               ms_per_step=round(dt / args.steps * 1e3, 3),
               higher_is_better=True, scaling="weak", vs_baseline=None,
               dtype="f64", data="synthetic (device-generated example.gmodel "
               "archives, float32)",
               config=dict(workload="configs[3]: %d tscrunched archives/GPU x "
                           "%dch x %dbin, ppalign iteration (phase+DM fit + "
                           "weighted rotate-and-sum)" % (args.nsub, nchan,
                                                          nbin),
                           nsub_per_gpu=args.nsub, nchan=nchan, nbin=nbin,
                           fit="align", parallelism="dp%d" % world, launcher=LAUNCHER),
               roofline=roof, solver_fp64=solver, kernels=kernels, cpu_baseline=None,
               template_peak=float(torch.as_tensor(m).abs().max()), **fitstats)
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        out["cpu_baseline"], out["parity"] = _align_cpu_baseline(
            b, noise, model0, min(args.cpu_sample, count), step, R, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.barrier()


def _align_cpu_baseline(b, noise, model0, nsamp, step, R, dev):
    """The oracle's align_archives (ppalign.py:65-257 restated) for ONE
    iteration over the first `nsamp` archives, one core, from the same
    initial template; parity: the device iteration over the same archives
    (its normalised template) against the oracle's."""
    import torch
    from types import SimpleNamespace
    import oracle.ppfit_oracle as O
    from threadpoolctl import threadpool_limits
    from pulseportraiture_amd import synth
    data = b["data"][:nsamp].double().cpu().numpy()
    nchan, nbin = data.shape[1:]
    arch = [SimpleNamespace(
        subints=data[i][None, None], weights=np.ones((1, nchan)),
        freqs=b["freqs"][None], Ps=b["P"][i:i + 1],
        SNRs=np.ones((1, 1, nchan)), noise_stds=noise[i][None, None],
        ok_isubs=[0], ok_ichans=[np.arange(nchan)], DM=synth.DM0, dmc=0,
        nbin=nbin) for i in range(nsamp)]
    mdl = SimpleNamespace(masks=np.ones((1, 1, nchan, nbin)),
                          subints=model0[None, None], freqs=b["freqs"][None],
                          ok_ichans=[np.arange(nchan)])
    with threadpool_limits(1):
        t0 = time.perf_counter()
        ref, _ = O.align_archives(arch, mdl, fit_dm=True, niter=1)
        dt = time.perf_counter() - t0
    Rs = SimpleNamespace(**{k: v[:nsamp] for k, v in R.__dict__.items()
                            if not k.startswith("_") and k != "n"})
    Rs.n = nsamp
    got = step(model0, R=Rs, timed=False).cpu().numpy()
    scale = float(np.abs(ref[0]).max())
    dev_max = float(np.abs(got - ref[0]).max()) / scale
    base = dict(value=nsamp / dt, unit="archive-iterations/s", cores=1,
                kind="port",
                sample="%d archives of %dch x %dbin, one oracle "
                       "align_archives iteration (guess + phase/DM fit + "
                       "rotate-and-sum per archive), %.1f s" %
                       (nsamp, nchan, nbin, dt),
                cpu_model=_cpu_model(), nproc=os.cpu_count())
    parity = dict(n=nsamp, max_abs_diff_over_peak=dev_max,
                  ok=bool(dev_max < 1e-6),
                  against="oracle align_archives iteration on the "
                          "cpu_baseline archives (same initial template)")
    return base, parity


class _Epoch(object):
    """psrchive.MJD stand-in for the in-memory archives (the TOA epoch
    arithmetic get_TOAs does: + seconds, in_days, intday, fracday)."""

    def __init__(self, days=0.0):
        self.days = float(days)

    def __add__(self, other):
        return _Epoch(self.days + (other.days if isinstance(other, _Epoch)
                                   else other / 86400.0))

    def in_days(self):
        return self.days

    def intday(self):
        return int(self.days)

    def fracday(self):
        return self.days - int(self.days)


def _host_rows(data, pinned):
    """The archive's amplitudes in host memory: pageable (as a plain
    load_data gives them) or, with --pinned, page-locked (a loader reading
    straight into pinned buffers)."""
    from pulseportraiture_amd import engine
    if not pinned:
        return data.cpu().numpy()
    out = engine.pinned_host_array(tuple(data.shape), np.float32)
    out[...] = data.cpu().numpy()
    return out


def _write_psrfits(path, b, f, per):
    """One synthetic archive as a 16-bit fold-mode PSRFITS file (device
    quantisation: per-profile offset = midrange, scale = half-range /
    32767, as psrfits.quantize)."""
    import torch
    from pulseportraiture_amd import psrfits, synth
    x = b["data"].double()
    lo, hi = x.amin(dim=-1), x.amax(dim=-1)
    offs = ((lo + hi) / 2).float()
    scl = ((hi - lo) / 2 / 32767.0).clamp_min(1e-30).float()
    q = torch.round((x - offs.double()[..., None]) / scl.double()[..., None])
    q = q.clamp(-32768, 32767).to(torch.int16).cpu().numpy()
    n, nchan, nbin = q.shape
    psrfits.write_psrfits(
        path, q[:, None], scl.cpu().numpy(), offs.cpu().numpy(),
        np.tile(b["freqs"], (n, 1)), np.ones((n, nchan)), b["P"],
        30.0 + 60.0 * np.arange(n), np.full(n, 60.0), stt_imjd=57000 + f,
        npol=1, pol_type="AA+BB", telescope="GBT", frontend="fake_rx",
        backend="fake_be", source="J1234-5678", dm=synth.DM0)
    return path


def bench_gettoas(args):
    """End-to-end GetTOAs.get_TOAs (pptoas.py:161-792) over in-memory
    archives (float32 amplitudes in host memory, as load_data hands them
    over): per archive the host batch build, the pinned double-buffered
    upload on the copy stream, ONE ppf_fit_batch on the worker stream and
    the per-sub-int bookkeeping into TOA objects, pipelined across archives.
    One step = one get_TOAs call over every archive; the rate includes the
    PCIe upload and the host bookkeeping, so it is not
    the kernel-path `value` of the headline line.  N > 1: the archives are
    sharded over the ranks (GetTOAs' archive mode: a rank builds, loads and
    fits only its own contiguous block of archives; the per-archive results
    are gathered at the end; strong scaling: the archive set is fixed).
    load_data is a dict lookup here: no PSRCHIVE read cost is charged."""
    import tempfile
    import torch
    from pulseportraiture_amd import dist, engine, pptoas, synth
    from pulseportraiture_amd.pplib import DataBunch, get_bin_centers
    rank, world, local = dist.init(args.dist_backend)
    dev = torch.device("cuda", local)
    nchan, nbin, per = args.nchan, args.nbin, args.arch_nsub
    nfile = max(1, args.nsub // per)
    files = {}
    a0, na = dist.shard(nfile, rank, world) if nfile >= world else (0, nfile)
    tmp = tempfile.mkdtemp()
    for f in range(nfile):
        name = "synthetic_%04d.fits" % f
        if not a0 <= f < a0 + na:
            files[name] = None          # another rank's archive: never loaded
            continue
        b = synth.make_batch(per, nchan, nbin, first=f * per, dev=dev)
        if args.psrfits:
            files[name] = _write_psrfits(os.path.join(tmp, name), b, f, per)
            del b
            continue
        noise = engine.noise_rows(b["data"]).cpu().numpy()
        snrs = (b["data"].amax(dim=-1).double().cpu().numpy() / noise * 3.0)
        files[name] = DataBunch(
            arch=None, backend="fake_be", backend_delay=0.0, bw=800.0,
            doppler_factors=np.ones(per), DM=synth.DM0, dmc=0,
            epochs=[_Epoch(57000.0 + f + i * 60.0 / 86400.0)
                    for i in range(per)],
            filename=name, flux_prof=np.array([]),
            freqs=np.tile(b["freqs"], (per, 1)), frontend="fake_rx",
            integration_length=60.0 * per, masks=None, nbin=nbin,
            nchan=nchan, noise_stds=noise[:, None], npol=1, nsub=per,
            nu0=1500.0, ok_ichans=[np.arange(nchan)] * per,
            ok_isubs=np.arange(per), parallactic_angles=np.zeros(per),
            phases=get_bin_centers(nbin), prof=None, prof_noise=1.0,
            prof_SNR=100.0, Ps=b["P"], SNRs=snrs[:, None],
            source="J1234-5678", state="Intensity",
            subints=_host_rows(b["data"], args.pinned)[:, None],
            subtimes=[60.0] * per,
            telescope="GBT", telescope_code="1", weights=np.ones((per, nchan)))
        del b
    torch.cuda.synchronize(dev)
    def load(fn, **kw):
        if files[fn] is None:
            raise AssertionError("rank %d loaded another rank's archive %s"
                                 % (rank, fn))
        return files[fn]
    if not args.psrfits:
        pptoas.load_data = load
        pptoas._MJD = _Epoch
    gm = synth.write_gmodel(os.path.join(tmp, "example.gmodel"))
    meta = os.path.join(tmp, "meta.txt")
    with open(meta, "w") as fh:
        fh.write("".join((files[n] if args.psrfits and files[n] else n) + "\n"
                         for n in files))

    def step():
        gt = pptoas.GetTOAs(meta, gm, quiet=True)
        gt.get_TOAs(quiet=True)
        return gt

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    dist.barrier()
    from pulseportraiture_amd import timeline
    if args.timeline:
        timeline.ENABLED = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        timeline.dump()
        ts = time.perf_counter()
        gt = step()
    torch.cuda.synchronize(dev)
    te = time.perf_counter()
    dist.barrier()
    dt = dist.max_over_ranks(time.perf_counter() - t0, dev)
    if args.timeline and rank == 0:
        spans = timeline.dump()
        summ = {}
        for name, th, a, b, c in spans:
            e = summ.setdefault(name, dict(count=0, total_ms=0.0, cpu_ms=0.0,
                                           threads=[]))
            e["count"] += 1
            e["total_ms"] += (b - a) * 1e3
            e["cpu_ms"] += c * 1e3
            if th not in e["threads"]:
                e["threads"].append(th)
        with open(args.timeline, "w") as fh:
            json.dump(dict(step_ms=(te - ts) * 1e3, ntoa=nfile * per,
                           stages={k: dict(v, mean_ms=v["total_ms"] /
                                           v["count"],
                                           mean_cpu_ms=v["cpu_ms"] /
                                           v["count"])
                                   for k, v in sorted(summ.items())},
                           spans=[(n, th, round((a - ts) * 1e3, 3),
                                   round((b - ts) * 1e3, 3),
                                   round(c * 1e3, 3))
                                  for n, th, a, b, c in spans]), fh, indent=1)
    ntoa = nfile * per
    out = dict(metric="GetTOAs end-to-end sub-int TOAs/sec (phase+DM, "
                      "%dch×%dbin, host archives, PCIe + bookkeeping "
                      "included)" % (nchan, nbin),
               value=round(ntoa * args.steps / dt, 2), unit="TOAs/s",
               n_gpus=world, steps=args.steps, warmup=args.warmup,
               ms_per_step=round(dt / args.steps * 1e3, 3),
               higher_is_better=True, scaling="strong", vs_baseline=None,
               dtype="f64", data="synthetic (device-generated example.gmodel "
               "archives %s)" % (
                   "written as 16-bit fold-mode PSRFITS files and read "
                   "through the PSRFITS fast path" if args.psrfits else
                   "held in %s host memory as float32" % (
                       "page-locked" if args.pinned else "pageable")),
               config=dict(workload="configs[1]-shape archives: %d x %d "
                           "sub-ints x %dch x %dbin through GetTOAs.get_TOAs"
                           % (nfile, per, nchan, nbin), nfile=nfile,
                           host_memory="pinned" if args.pinned else "pageable",
                           nsub_per_archive=per, nchan=nchan, nbin=nbin,
                           fit="gettoas", parallelism="dp%d" % world, launcher=LAUNCHER,
                           sharding="archives" if nfile >= world and
                           world > 1 else "sub-ints" if world > 1 else None,
                           load_data="PSRFITS fast path (psrfits.load_data:"
                           " mmap, pinned copy of the DATA bytes, device "
                           "unpack + baseline + noise; files in the page "
                           "cache)" if args.psrfits else
                           "in-memory dict lookup (no PSRCHIVE "
                           "read cost charged)"),
               toas=len(gt.TOA_list), host_gb=round(
                   nfile * per * nchan * nbin * (2 if args.psrfits else 4)
                   / 1e9, 2),
               roofline=None, cpu_baseline=None)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.barrier()


def bench_single(args):
    """Single-call latency of the drop-in APIs, one sub-integration per call
    as ppgauss.py:318 (fit_portrait), DataPortrait (pplib.py:362-370,
    rotate_data) and scripts calling fit_portrait_full directly use them:
    each call uploads its host arrays, runs the batch-of-one device path and
    returns host results (synchronised).  Shapes: configs[0]'s 64 x 512 and
    configs[1]'s 512 x 2048.  Beside each, the oracle's time for the same
    call on one core (its fit_portrait_full / fit_portrait / rotate_data
    restatements of the reference)."""
    import torch
    import oracle.ppfit_oracle as O
    from threadpoolctl import threadpool_limits
    from pulseportraiture_amd import pplib, pptoaslib, synth
    dev = torch.device("cuda", 0)
    calls = {}
    for nchan, nbin in ((64, 512), (512, 2048)):
        b = synth.make_batch(1, nchan, nbin, dev=dev)
        data = b["data"][0].cpu().numpy()
        model, freqs, P = b["model"], b["freqs"], float(b["P"][0])
        nu_fit = pplib.guess_fit_freq(freqs)
        init = [float(b["phi_true"][0]) + 1e-3, synth.DM0, 0.0, 0.0, 0.0]
        init[0] = float(O.phase_transform(init[0], synth.DM0, 1500.0, nu_fit,
                                          P, mod=True))
        errs = O.noise_ps(data.astype(np.float64))
        ffl = [1, 1, 0, 0, 0]
        api = {
            "fit_portrait_full": (
                lambda: pptoaslib.fit_portrait_full(
                    data, model, init, P, freqs, [nu_fit] * 3, [None] * 3,
                    errs, ffl, log10_tau=False),
                lambda: O.fit_portrait_full(
                    data.astype(np.float64), model, init, P, freqs,
                    [nu_fit] * 3, [None] * 3, errs, ffl, log10_tau=False)),
            "fit_portrait": (
                lambda: pplib.fit_portrait(data, model, init[:2], P, freqs,
                                           nu_fit, None, errs),
                lambda: O.fit_portrait(data.astype(np.float64), model,
                                       init[:2], P, freqs, nu_fit, None,
                                       errs)),
            "rotate_data": (
                lambda: pplib.rotate_data(data, 0.1, synth.DM0, P, freqs,
                                          1500.0),
                lambda: O.rotate_data(data.astype(np.float64), 0.1,
                                      synth.DM0, P, freqs, 1500.0)),
        }
        for name, (gpu, cpu) in api.items():
            for _ in range(max(2, args.warmup)):
                gpu()
            torch.cuda.synchronize(dev)
            ts = []
            for _ in range(max(5, args.steps)):
                t0 = time.perf_counter()
                gpu()
                ts.append(time.perf_counter() - t0)
            with threadpool_limits(1):
                cpu()
                tc = []
                for _ in range(3):
                    t0 = time.perf_counter()
                    cpu()
                    tc.append(time.perf_counter() - t0)
            calls["%s_%dx%d" % (name, nchan, nbin)] = dict(
                gpu_ms_median=round(1e3 * float(np.median(ts)), 3),
                gpu_ms_min=round(1e3 * float(np.min(ts)), 3),
                cpu_oracle_ms_median=round(1e3 * float(np.median(tc)), 3),
                speedup=round(float(np.median(tc) / np.median(ts)), 2))
    key = "fit_portrait_full_64x512"
    out = dict(metric="single-call latency of the drop-in APIs (one "
                      "sub-integration per call, host arrays in and out)",
               value=calls[key]["gpu_ms_median"], unit="ms",
               n_gpus=1, steps=max(5, args.steps), warmup=max(2, args.warmup),
               higher_is_better=False, scaling=None, vs_baseline=None,
               dtype="f64", data="synthetic (example.gmodel portraits + "
               "white noise; float32 amplitudes)",
               config=dict(workload="fit_portrait_full / fit_portrait / "
                           "rotate_data, one call per sub-int at 64x512 and "
                           "512x2048 (value: fit_portrait_full 64x512)",
                           fit="single"),
               calls=calls, roofline=None,
               cpu_baseline=dict(value=calls[key]["cpu_oracle_ms_median"],
                                 unit="ms", cores=1, kind="port",
                                 sample="the oracle's fit_portrait_full of "
                                        "the same 64x512 sub-int, median of "
                                        "3 calls"))
    print(json.dumps(out), flush=True)


def self_launch(args):
    """`python bench.py --gpus N` (N > 1) with no launcher: start the N ranks
    here (one child process per GPU, RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set, dist.launch_local) and return their exit status; rank 0's
    JSON line is forwarded.  This parent never touches the GPU (counting
    devices does not initialise HIP) and never re-execs.  With fewer visible
    devices than ranks (the one-GPU gloo rehearsal) ranks share devices
    round-robin; RCCL needs one device per rank, so that raises for nccl."""
    import torch
    from pulseportraiture_amd import dist
    ndev = torch.cuda.device_count()
    if ndev < args.gpus and args.dist_backend == "nccl":
        print("error: --gpus %d with %d visible devices (RCCL needs one "
              "device per rank)" % (args.gpus, ndev), file=sys.stderr)
        return 2
    local = (lambda r: r % ndev) if 0 < ndev < args.gpus else None
    return dist.launch_local(os.path.abspath(__file__), sys.argv[1:],
                             args.gpus, local_ranks=local)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    if args.fit == "single":
        return bench_single(args)
    if args.fit == "align":
        return bench_align(args)
    if args.fit == "gettoas":
        if args.nsub == 10000:
            args.nsub = 2048            # 8.6 GB of host archives
        return bench_gettoas(args)
    import torch
    from pulseportraiture_amd import _lib, dist, engine, synth
    from pulseportraiture_amd.pplib import guess_fit_freq
    rank, world, local = dist.init(args.dist_backend)
    if world != args.gpus and rank == 0:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world),
              file=sys.stderr)
    dev = torch.device("cuda", local)
    total = args.nsub * world
    first, count = dist.shard(total, rank, world)
    nchan, nbin = args.nchan, args.nbin
    nharm = nbin // 2 + 1

    # ---- resident inputs (untimed) ------------------------------------------
    # fit modes: C3 injects tau = 2e-3 rot at 1500 MHz,
    # C5 tau = 5e-3 rot at 600 MHz over 400-800 MHz; alpha = -4, and the
    # GetTOAs guesses tau = 1/nbin (log10), alpha = -4 (pptoas.py:467-492)
    FIT = {"phase+DM": dict(flags=[1, 1, 0, 0, 0], band=(1100.0, 800.0),
                            tau=0.0, nu_tau=None, cfg=1),
           "full": dict(flags=[1, 1, 1, 1, 1], band=(1100.0, 800.0),
                        tau=2e-3, nu_tau=1500.0, cfg=2),
           "scat": dict(flags=[1, 1, 0, 1, 1], band=(400.0, 400.0),
                        tau=5e-3, nu_tau=600.0, cfg=4)}[args.fit]
    scat_fit = FIT["tau"] > 0.0
    batch = synth.make_batch(count, nchan, nbin, first=first, dev=dev,
                             lo=FIT["band"][0], bw=FIT["band"][1],
                             tau=FIT["tau"], nu_tau=FIT["nu_tau"])
    data = batch["data"]
    f64 = torch.float64
    model_t = torch.as_tensor(batch["model"], dtype=f64, device=dev)
    freqs_t = torch.as_tensor(np.tile(batch["freqs"], (count, 1)), dtype=f64,
                              device=dev)
    P_t = torch.as_tensor(batch["P"], dtype=f64, device=dev)
    init = np.zeros((count, 5))
    init[:, 1] = synth.DM0                       # DM_guess = DM_stored
    if scat_fit:
        init[:, 3] = np.log10(1.0 / nbin)
        init[:, 4] = synth.GMODEL_ALPHA
    init_t = torch.as_tensor(init, dtype=f64, device=dev)
    flags_t = torch.tensor(FIT["flags"], dtype=torch.int32,
                           device=dev).repeat(count, 1)
    nu_fit = guess_fit_freq(batch["freqs"])      # pptoas.py:442
    nu_fits_t = torch.full((count, 3), nu_fit, dtype=f64, device=dev)
    nu_outs_t = torch.full((count, 3), float("nan"), dtype=f64, device=dev)
    gw_t = torch.ones((count, nchan), dtype=f64, device=dev)
    gdm_t = torch.full((count,), synth.DM0, dtype=f64, device=dev)
    mask_t = None
    if args.zap_frac > 0.0:      # the same channels zapped in every sub-int
        zrng = np.random.default_rng(20250217)
        keep = np.ones(nchan, np.uint8)
        keep[zrng.choice(nchan, int(round(args.zap_frac * nchan)),
                         replace=False)] = 0
        mask_t = torch.as_tensor(np.tile(keep, (count, 1)), device=dev)
    lib = _lib.load()
    ctx = _lib.context(dev.index)
    lib.ppf_set_profiling(ctx, 1)
    ws = None
    if args.passes is None:
        args.passes = 24 if args.fit == "phase+DM" else 1
    n_x_all = count if scat_fit else 0       # X slots: scattering fits only
    if args.chunk is None:
        # one ppf_fit_batch call per GPU per step, unless the cross spectrum
        # of the scattering fits (nchan nharm 16 B per sub-int) would pass
        # ~150 GB of the 288 GB HBM
        args.chunk = count if not scat_fit else max(1, min(
            count, int(150e9 // (nchan * nharm * 16))))
    chunks = [(c0, min(count, c0 + args.chunk))
              for c0 in range(0, count, args.chunk)]

    def step():
        nonlocal ws
        for _ in range(args.passes):
            outs = []
            for c0, c1 in chunks:
                sl = slice(c0, c1)
                res = engine.fit_batch(
                    data[sl], model_t, freqs_t[sl], P_t[sl], init_t[sl],
                    flags_t[sl], nu_fits=nu_fits_t[sl], nu_outs=nu_outs_t[sl],
                    log10_tau=scat_fit,
                    guess=True, guess_weights=gw_t[sl], guess_DM=gdm_t[sl],
                    guess_Ns=100,
                    chan_mask=None if mask_t is None else mask_t[sl],
                    dev=dev, workspace=ws,
                    n_x=(c1 - c0) if n_x_all else 0, no_hcut=args.no_hcut,
                    solver=args.solver, mom_x=MOMX[args.mom_x],
                    max_workspace=1 << 62)
                ws = res["workspace"]
                outs.append(res["results"])
            results = torch.cat(outs, 0)
        return dist.allgather_rows(results, total, world)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        last = step()
    torch.cuda.synchronize(dev)
    dist.barrier()
    dt = time.perf_counter() - t0
    dt = dist.max_over_ranks(dt, dev)

    # ---- per-kernel times of the timed region (HIP events on the stream) ---
    ncalls = min(256, len(chunks) * args.steps * args.passes)
    hist = np.zeros((ncalls, 4))
    got = lib.ppf_stage_ms_history(ctx, ncalls, hist.ctypes.data)
    stage_ms = hist[:got].sum(axis=0)
    khist = np.zeros((ncalls, 2))
    kgot = lib.ppf_kernel_ms_history(ctx, ncalls, khist.ctypes.data)
    kern_ms = khist[:kgot].sum(axis=0)
    phist = np.zeros((ncalls, 2))
    pgot = lib.ppf_pass_ms_history(ctx, ncalls, phist.ctypes.data)
    pass_ms, pass_launches = phist[:pgot].sum(axis=0)
    # solver kernels: [k_tr_mom ms, launches, k_tr_step ms, launches,
    # k_postfit ms, launches] summed over the calls
    shist = np.zeros((ncalls, 6))
    sgot = lib.ppf_solver_ms_history(ctx, ncalls, shist.ctypes.data)
    solv_ms = shist[:max(sgot, 0)].sum(axis=0)
    res_np = last.cpu().numpy()
    I = _lib.RESULT_INDEX
    nfev = res_np[:, I["nfeval"]]
    npass = res_np[:, I["npass"]]
    status = res_np[:, I["status"]].astype(int)
    # the event ring holds the last `ncalls` ppf_fit_batch calls
    steps_subints = count * ncalls // len(chunks)
    mine = slice(first, first + count) if world > 1 else slice(None)
    mean_passes = float(npass[mine].mean())
    mean_nfev = float(nfev[mine].mean())
    # ALGORITHMIC bytes per sub-integration:
    #  k_xmom_g (first, full moment pass): read the f32 rows, the channel
    #   derivatives dphi (2 f64); write 32 complex moments, the 4 channel
    #   scalars and the centre residual per channel.  The model spectra
    #   (nchan nharm 16 B) are read once per launch.
    #  k_dsum_w: read the f32 rows; write the per-block guess profiles.
    nblkd = (nchan + 127) // 128
    xmom_unit = nchan * nbin * 4 + nchan * 16 + nchan * (32 * 16 + 4 * 8 + 8)
    dsum_unit = nchan * nbin * 4 + nblkd * nbin * 8 + nblkd * 16
    #  k_xspec_w (scattering fits: the cross spectrum X streamed by every
    #   evaluation): read the rows, write X (complex128) and 4 scalars/channel
    #   X is written only below the harmonic cutoff of each aligned
    #   64-channel group (k_model_cut, |M_k|^2 > 1e-28 max |M|^2; DESIGN.md
    #   section 3), so the X bytes count those harmonics
    mp = np.abs(np.fft.rfft(np.asarray(batch["model"], dtype=np.float64),
                            axis=1)) ** 2
    mp[:, 0] = 0.0
    above = mp > 1e-28 * mp.max(axis=1, keepdims=True)
    kc = np.where(above.any(axis=1),
                  nharm - np.argmax(above[:, ::-1], axis=1), 1)
    kw = np.array([kc[g:g + 64].max() for g in range(0, nchan, 64)])
    xh = int(sum(kw[i] * min(64, nchan - 64 * i) for i in range(len(kw))))
    xspec_unit = nchan * nbin * 4 + xh * 16 + 4 * nchan * 8
    L2N = (nbin // 4).bit_length()
    kern = {
        "dsum": dict(name="k_dsum_w" if (nbin & (nbin - 1)) == 0 else "k_dsum_wn",
                     ms=kern_ms[1], unit=dsum_unit,
                     bytes=steps_subints * dsum_unit),
    }
    # the library's MOM_X rule (ppf_api.cpp fit_layout): X moments when asked,
    # or with the guess at nbin 2048 unless the fused pass is forced
    momx_used = not scat_fit and (args.mom_x == "x" or (
        args.mom_x == "auto" and nbin == 2048))
    # the wave-FFT kernels take power-of-two nbin in [256, 2048]; other
    # lengths (the mixed-radix 1000, 1536, ...) run the block-FFT spectrum
    # pass, which writes every harmonic of X, and k_moments
    wave = (nbin & (nbin - 1)) == 0 and 256 <= nbin <= 2048
    if not wave and not scat_fit:
        # nbin / 2 not a power of two, <= 1024: the wave-per-row mixed-radix
        # pass k_xspec_wm, which writes X below the cutoffs (like
        # k_xspec_w); longer rows: the block-FFT k_xspec, every harmonic
        # (odd nbin < 1024 too, rows as nbin complex points; longer odd rows
        # on the block-FFT pass)
        wm = (nbin % 2 == 0 and nbin // 2 <= 1024 and
              (nbin & (nbin - 1)) != 0) or (nbin % 2 == 1 and nbin < 1024)
        xfull = nchan * nbin * 4 + (xh if wm else nchan * nharm) * 16 + 4 * nchan * 8
        kern["xspec"] = dict(name=("k_xspec_wo" if nbin % 2 else "k_xspec_wm") if wm
                             else "k_xspec (block FFT)",
                             ms=stage_ms[1], unit=xfull,
                             bytes=steps_subints * xfull +
                             ncalls * nchan * nharm * 16)
        # (16 moments per channel about its band centre, and the centre:
        # ppf_api.cpp PPF_MOM16_BLOCK)
        mu = xh * 16 + nchan * 16 + nchan * (16 * 16 + 8 + 8)
        kern["moments"] = dict(name="k_moments", ms=kern_ms[0], unit=mu,
                               bytes=steps_subints * mu)
    elif scat_fit or momx_used:
        # 1024-point rows: k_xspec_w2 (the one-exchange wave FFT) unless
        # PPF_XSPEC2=0 selects k_xspec_w
        xname = ("k_xspec_w2<0>" if L2N == 10 and
                 os.environ.get("PPF_XSPEC2", "1") != "0"
                 else "k_xspec_w<%d, 0>" % L2N)
        kern["xspec"] = dict(name=xname, ms=stage_ms[1],
                             unit=xspec_unit,
                             bytes=steps_subints * xspec_unit +
                             ncalls * nchan * nharm * 16)
        #  k_pass<true> (one trust-region evaluation per launch of every fit
        #   still iterating): read the fit's cut X (the same xh harmonics
        #   k_xspec_w wrote), write its per-channel stats (10 f64) and the
        #   block partials (21 f64 per 256 channels); |M|^2 of the cut
        #   harmonics once per launch (shared by the batch: L2/MALL)
        nblkp = (nchan + 255) // 256
        pass_unit = xh * 16 + nchan * 80 + nblkp * 21 * 8
        evals = steps_subints * mean_passes
        kern["pass"] = dict(name="k_pass<true>", ms=pass_ms, unit=pass_unit,
                            launches=int(pass_launches),
                            bytes=evals * pass_unit + pass_launches * xh * 8)
    if momx_used and wave:
        #  k_moments (first launch: every sub-int): read X below the cutoff
        #   and dphi, write 16 complex moments about each channel band's
        #   centre (mom16, the X-moment path), the centre residual and the
        #   band centre
        mu = xh * 16 + nchan * 16 + nchan * (16 * 16 + 8 + 8)
        kern["moments"] = dict(name="k_moments", ms=kern_ms[0], unit=mu,
                               bytes=steps_subints * mu)
    elif not scat_fit and wave:
        kern["xmom"] = dict(name="k_xmom_g<%d, 0, true, true>" % L2N,
                            ms=kern_ms[0], unit=xmom_unit,
                            bytes=steps_subints * xmom_unit +
                            ncalls * nchan * nharm * 16)
    dom = max(kern, key=lambda k: kern[k]["ms"])
    dk = kern[dom]
    achieved = dk["bytes"] / (dk["ms"] / 1e3) / 1e9
    # HBM traffic per launch from the PMC passes (profiles/pmc_reduce.py):
    # measured bytes per unit x the units one launch processes
    nlaunch = dk.get("launches", ncalls)
    units_launch = (steps_subints if "launches" not in dk else
                    steps_subints * mean_passes) / nlaunch
    traffic = None
    # (the PMC / SQ summaries are of the default, cut configuration of this
    # fit mode, and apply only at the shape they were collected on)
    shape_tag = "%dch x %dbin" % (nchan, nbin)

    def _same_shape(m):
        return shape_tag in str((m.get("source") or {}).get("bench", ""))
    # summary entry: the fit mode, or "mode@nbin" for non-power-of-two nbin
    # (profiles/pmc_reduce.py, fp64_reduce.py)
    mkey = args.fit if nbin & (nbin - 1) == 0 else "%s@%d" % (args.fit, nbin)
    if os.path.exists(args.pmc) and not args.no_hcut:
        pm = json.load(open(args.pmc)).get("modes", {}).get(mkey, {})
        pk = pm.get("kernels", {}).get(dom) if _same_shape(pm) else None
        if pk:
            traffic = round(pk["hbm_bytes"] * units_launch)
    roof = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS,
                unit="GB/s", frac=round(achieved / HBM_PEAK_GBS, 4),
                traffic=traffic, kernel=dk["name"],
                algorithmic_bytes_per_launch=dk["bytes"] / nlaunch,
                algorithmic_bytes_per_unit=dk["unit"],
                avg_launch_ms=round(dk["ms"] / nlaunch, 4),
                launches=int(nlaunch), units_per_launch=units_launch)
    # fp64 issue roofline of the same kernel: flops per unit from the SQ
    # counter passes (profiles/fp64_reduce.py: f64 VALU add/mul/fma/trans x 64
    # lanes, fma x 2, + 512 per f64 MFMA MOP) x the units of one launch / the
    # launch's event-timed duration, against the fp64 peak
    fp64 = None
    fpath = os.path.join(ROOT, "profiles", "fp64_summary.json")
    if os.path.exists(fpath) and not args.no_hcut:
        fm = json.load(open(fpath)).get("modes", {}).get(mkey, {})
        fk = fm.get("kernels", {}).get(dom) if _same_shape(fm) else None
        if fk:
            tf = fk["flops_per_unit"] * units_launch / (dk["ms"] / nlaunch / 1e3) / 1e12
            fp64 = dict(bound="fp64", achieved=round(tf, 2), peak=FP64_PEAK_TF,
                        unit="TFLOP/s", frac=round(tf / FP64_PEAK_TF, 4),
                        flops_per_unit=round(fk["flops_per_unit"]),
                        valu_f64_per_unit=round(fk["valu_f64_per_unit"]),
                        mfma_f64_per_unit=round(fk["mfma_f64_per_unit"], 1),
                        valu_active_per_wave=fk.get("valu_active_per_wave"),
                        clock_ghz=fk.get("clock_ghz"),
                        source=os.path.relpath(fpath, ROOT))
            # VALU issue floor of one launch: 4 cycles per f64 and 2 per
            # other wave64 VALU instruction (MI355X: 16 f64 / 32 f32 lanes
            # per SIMD per clock) over the 1024 SIMDs at the clock the chip
            # held; the launch's measured time over it
            if fk.get("valu_all_per_unit") is not None and fk.get("clock_ghz"):
                v64 = fk["valu_f64_per_unit"]
                cyc = 4.0 * v64 + 2.0 * (fk["valu_all_per_unit"] - v64)
                floor_ms = units_launch * cyc / (1024 * fk["clock_ghz"] * 1e9) * 1e3
                fp64["issue_floor_ms"] = round(floor_ms, 4)
                fp64["issue_floor_frac"] = round(floor_ms / (dk["ms"] / nlaunch), 4)
                roof["issue_floor_ms"] = fp64["issue_floor_ms"]
                roof["issue_floor_frac"] = fp64["issue_floor_frac"]
                roof["valu_active_per_wave"] = fk.get("valu_active_per_wave")
    # fp64 utilisation of the SOLVER (north star: "fp64 VALU utilisation for
    # the solver"): the trust-region kernels of the fit mode, their f64
    # flops per unit from the same SQ counter passes (fp64_summary.json) x
    # the units of the timed calls / their HIP-event time.  Moment path
    # (phase+DM, align): k_tr_mom (every iteration of every fit from the
    # moments) + k_moments (the moment sets; for the fused path k_xmom_g
    # carries them and is priced above); scattering path: k_pass (the
    # objective / gradient / Hessian sums of every evaluation) + k_tr_step.
    # k_postfit (covariance, zero-covariance roots) is listed for both.
    solver = None
    if os.path.exists(fpath) and not args.no_hcut:
        fm = json.load(open(fpath)).get("modes", {}).get(mkey, {})
        fk = fm.get("kernels", {}) if _same_shape(fm) else {}
        parts = []
        if scat_fit:
            parts.append(("pass", "k_pass<true>", pass_ms,
                          steps_subints * mean_passes, pass_launches))
            parts.append(("tr_step", "k_tr_step", solv_ms[2], None, solv_ms[3]))
        else:
            parts.append(("tr_mom", "k_tr_mom", solv_ms[0], None, solv_ms[1]))
            if "moments" in kern:
                parts.append(("moments", "k_moments", kern["moments"]["ms"],
                              steps_subints, ncalls))
        parts.append(("postfit", "k_postfit", solv_ms[4], steps_subints,
                      solv_ms[5]))
        solver = _solver_fp64(fk, parts, nchan, 16 if (momx_used or not wave) else 32,
                              steps_subints * mean_nfev, fpath)
    names = ["model_rfft", "xspec", "guess", "solve"]
    stages = {n: round(float(stage_ms[i]), 3) for i, n in enumerate(names)}
    kernels = {k: dict(name=v["name"], total_ms=round(float(v["ms"]), 3),
                       launches=int(v.get("launches", ncalls)),
                       avg_launch_ms=round(float(v["ms"]) /
                                           max(1, v.get("launches", ncalls)), 4),
                       gbs=(None if not v["ms"] else
                            round(v["bytes"] / (v["ms"] / 1e3) / 1e9, 1)))
               for k, v in kern.items()}
    value = total * args.steps * args.passes / dt
    metric = METRIC if args.fit == "phase+DM" else (
        "subint portrait fits/sec (%s, %dch×%dbin) at 1/2/4/8 MI355X" %
        ("phi+DM+GM+tau+alpha" if args.fit == "full" else "phi+DM+tau+alpha",
         nchan, nbin))
    out = dict(metric=metric, value=round(value, 2), unit="subint-fits/s",
               n_gpus=world, steps=args.steps, warmup=args.warmup,
               ms_per_step=round(dt / args.steps * 1e3, 3),
               higher_is_better=True, scaling="weak", vs_baseline=None,
               dtype="f64", data="synthetic (device-generated example.gmodel "
               "portraits + white noise; float32 amplitudes)",
               config=dict(workload="configs[%d]: %d subints/GPU x %dch x "
                           "%dbin, %s wideband fit (GetTOAs fit stage: guess + fit + post-fit of HBM-resident sub-ints; --fit gettoas times the host path)%s" %
                           (FIT["cfg"], args.nsub, nchan, nbin, args.fit,
                            "" if not scat_fit else
                            ", injected tau %g rot at %g MHz" %
                            (FIT["tau"], FIT["nu_tau"])),
                           nsub_per_gpu=args.nsub, passes_per_step=args.passes,
                           fits_per_step=total * args.passes,
                           nchan=nchan, nbin=nbin, chunk=args.chunk,
                           harmonic_cutoff=not args.no_hcut,
                           solver=args.solver, mom_x=args.mom_x,
                           moments="cross spectrum (k_xspec_w + k_moments)"
                           if momx_used and wave else (
                               "fused pass (k_xmom_g)" if wave else
                               "cross spectrum (k_xspec_w%s + k_moments)" %
                               ("o" if nbin % 2 else "m")
                               if (nbin % 2 == 0 and nbin // 2 <= 1024 and
                                   (nbin & (nbin - 1))) or
                               (nbin % 2 == 1 and nbin < 1024) else
                               "cross spectrum (block FFT + k_moments)"),
                           zap_frac=args.zap_frac,
                           fit=args.fit, fit_flags=FIT["flags"],
                           parallelism="dp%d" % world, launcher=LAUNCHER),
               roofline=roof, fp64_roofline=fp64, solver_fp64=solver,
               stage_ms=stages, kernels=kernels,
               # algorithmic HBM bytes of the priced kernels per fit (the
               # guess pass, the spectrum / moment pass and, for scattering
               # fits, every streaming evaluation)
               bytes_per_fit=round(sum(float(v["bytes"]) for v in kern.values())
                                   / max(steps_subints, 1)),
               mean_passes_per_fit=round(mean_passes, 3),
               mean_evals_per_fit=round(mean_nfev, 3),
               fits_converged_frac=round(float(np.mean(
                   (status & 0xff) == 2)), 5),
               # the gathered result records of the last step (every sub-int
               # of every rank, global order): equal across world sizes
               # (tests/test_gpu_dist.py)
               results_sha256=hashlib.sha256(
                   np.ascontiguousarray(res_np).tobytes()).hexdigest())
    # sanity: fitted DM / phase agree with the injected truths
    if rank == 0:
        dm = res_np[:count, I["params"]][:, 1]
        dme = res_np[:count, I["param_errs"]][:, 1]
        pull = (dm - batch["DM_true"]) / dme
        out["dm_pull_rms"] = round(float(np.sqrt(np.mean(pull ** 2))), 3)
    if scat_fit and rank == 0:
        # log10 tau at the output reference frequency vs the injected truth
        pr = res_np[:count, I["params"]]
        pe = res_np[:count, I["param_errs"]]
        nuo = res_np[:count, I["nu_out"]][:, 2]
        truth = np.log10(FIT["tau"] * (nuo / FIT["nu_tau"]) ** synth.GMODEL_ALPHA)
        out["tau_pull_rms"] = round(float(np.sqrt(np.mean(
            ((pr[:, 3] - truth) / pe[:, 3]) ** 2))), 3)
        out["alpha_pull_rms"] = round(float(np.sqrt(np.mean(
            ((pr[:, 4] - synth.GMODEL_ALPHA) / pe[:, 4]) ** 2))), 3)
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        # scattering fits take ~10x longer on the CPU: a 12x smaller sample
        # (C5's 16384-channel fits ~30 s each: 48x smaller); the default
        # --cpu-sample 48 gives C3 4 and C5 1 one-core sub-ints, 192 gives
        # 16 and 4 (the evidence runs, tools/evid.sh)
        nsamp = min(args.cpu_sample if not scat_fit else
                    (max(4, args.cpu_sample // 12) if nchan * nbin <= 1 << 20
                     else max(1, args.cpu_sample // 48)), count)
        out["cpu_baseline"], oref = cpu_baseline(
            batch, nsamp, nchan, nbin, args.cpu_workers, mode=args.fit,
            flags=FIT["flags"], per_worker=4 if not scat_fit else 1)
        out["vs_cpu_baseline"] = round(value / out["cpu_baseline"]["value"],
                                       1)
        out["parity"] = parity_vs_oracle(res_np[:nsamp], oref, batch["P"],
                                         FIT["flags"])
        if "all_core" in oref:
            # and the all-core run's sub-ints (C5: 16 sub-ints, where one
            # single-core fit takes ~28 s)
            na = oref["n_all"]
            out["parity_all_core"] = parity_vs_oracle(
                res_np[:na], oref["all_core"], batch["P"], FIT["flags"])
    else:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.barrier()


if __name__ == "__main__":
    main()

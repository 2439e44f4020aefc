"""PSRCHIVE-free fast path from fold-mode PSRFITS files to the device.

SURVEY.md 8(f)3: the host must not starve the GPUs.  PSRCHIVE's load_data
(pplib.py:2749-2915) unpacks every sample to float on the host, removes the
baseline, pscrunches and computes noise and S/N per profile before anything
reaches the device.  Here the file is memory-mapped, only its headers are
parsed on the host, and the SUBINT table's raw DATA bytes (big-endian
integers, 2 B per sample for the usual 16-bit archives) go straight into
pinned staging buffers and over PCIe; the device then unpacks them
(DATA * DAT_SCL + DAT_OFFS in float32 arithmetic, as PSRCHIVE's FITS loader
does), sums the polarisations to total intensity, removes the baseline and
measures noise and S/N per channel (ppf_unpack_psrfits_batch, then
ppf_noise_batch).  The archive's rows stay in HBM for the fit.

This module is the FITS side: a minimal reader of the primary header and the
SUBINT / POLYCO binary tables (FITS 4.0 standard: 2880-byte blocks, 80-byte
header cards, big-endian binary tables), and a writer of the same subset
(tests, bench).  Fold-mode (OBS_MODE PSR/CAL) archives only; search-mode
data, FITS templates and PSRCHIVE's other formats stay with PSRCHIVE.

What is restated from PSRCHIVE's documented behaviour and NOT pinned to a
PSRCHIVE run (PSRCHIVE is absent from this image and the reference holds no
PSRFITS fixture):
  * the epoch of sub-int i is the start time plus OFFS_SUB (STT_IMJD,
    STT_SMJD, STT_OFFS, OFFS_SUB); PSRCHIVE's loader may further refer it to
    the folding predictor;
  * the folding period is the SUBINT PERIOD column when present, else the
    POLYCO table evaluated at the epoch (TEMPO polyco formula);
  * Doppler factors need an ephemeris: they are 1 (the TOAs are
    topocentric, as get_TOAs(bary=False) leaves them);
  * baseline removal: PSRCHIVE's default BaselineWindow (the minimum mean
    over a window of 15 % of the turn on the total profile of the sub-int,
    subtracted from every channel);
  * S/N per channel: the baseline-subtracted profile's sum over the
    on-pulse bins (outside the baseline window) / (sigma_off sqrt(n_on)).
"""
import mmap
import os
import threading

import numpy as np

BLOCK = 2880
_TFORM = {"L": (1, "u1"), "B": (1, "u1"), "I": (2, ">i2"), "J": (4, ">i4"),
          "K": (8, ">i8"), "A": (1, "S1"), "E": (4, ">f4"), "D": (8, ">f8"),
          "C": (8, ">c8"), "M": (16, ">c16")}


def _parse_value(v):
    v = v.strip()
    if v.startswith("'"):
        end = v.find("'", 1)
        while end + 1 < len(v) and v[end + 1] == "'":      # '' escape
            end = v.find("'", end + 2)
        return v[1:end].replace("''", "'").rstrip()
    if "/" in v:
        v = v.split("/", 1)[0].strip()
    if v in ("T", "F"):
        return v == "T"
    try:
        return int(v)
    except ValueError:
        pass
    try:
        return float(v.replace("D", "E"))
    except ValueError:
        return v


def _read_header(buf, off):
    """(dict of cards, offset of the data) of the HDU header at off."""
    hdr = {}
    while True:
        if off + BLOCK > len(buf):
            raise ValueError("truncated FITS header")
        block = bytes(buf[off:off + BLOCK]).decode("ascii", "replace")
        off += BLOCK
        for i in range(0, BLOCK, 80):
            card = block[i:i + 80]
            key = card[:8].strip()
            if key == "END":
                return hdr, off
            if card[8:10] == "= " and key:
                hdr[key] = _parse_value(card[10:])


def _data_bytes(hdr):
    naxis = int(hdr.get("NAXIS", 0))
    if naxis == 0:
        return 0
    n = 1
    for i in range(1, naxis + 1):
        n *= int(hdr["NAXIS%d" % i])
    n = abs(int(hdr.get("BITPIX", 8))) // 8 * int(hdr.get("GCOUNT", 1)) * \
        (int(hdr.get("PCOUNT", 0)) + n)
    return (n + BLOCK - 1) // BLOCK * BLOCK


class Table(object):
    """A binary-table HDU: header cards and column accessors (views into
    the mapped file)."""

    def __init__(self, hdr, buf, off):
        self.header = hdr
        self.nrows, self.rowbytes = int(hdr["NAXIS2"]), int(hdr["NAXIS1"])
        self._buf, self._off = buf, off
        self.columns = {}
        pos = 0
        for i in range(1, int(hdr["TFIELDS"]) + 1):
            form = str(hdr["TFORM%d" % i]).strip()
            j = 0
            while j < len(form) and form[j].isdigit():
                j += 1
            rep = int(form[:j]) if j else 1
            code = form[j]
            size, dt = _TFORM[code]
            name = str(hdr.get("TTYPE%d" % i, "COL%d" % i)).strip()
            dim = hdr.get("TDIM%d" % i)
            self.columns[name] = (pos, rep, dt, code, dim)
            pos += rep * size
        if pos != self.rowbytes:
            raise ValueError("binary table row size mismatch")

    def raw(self):
        """The table as a [nrows, rowbytes] uint8 view of the mapped file."""
        return np.frombuffer(self._buf, dtype=np.uint8,
                             count=self.nrows * self.rowbytes,
                             offset=self._off).reshape(self.nrows,
                                                       self.rowbytes)

    def has(self, name):
        return name in self.columns

    def column(self, name):
        """[nrows, repeat] array of a column (a strided view, big-endian;
        character columns as str)."""
        pos, rep, dt, code, _ = self.columns[name]
        raw = self.raw()
        if code == "A":
            return [bytes(r[pos:pos + rep]).decode("ascii", "replace").rstrip()
                    for r in raw]
        size = _TFORM[code][0]
        v = raw[:, pos:pos + rep * size]
        return np.ascontiguousarray(v).view(dt).reshape(self.nrows, rep)

    def column_bytes(self, name):
        """(strided uint8 view [nrows, nbytes], element dtype) of a column:
        the DATA bytes as they sit in the file, for the device unpack."""
        pos, rep, dt, code, _ = self.columns[name]
        size = _TFORM[code][0]
        return self.raw()[:, pos:pos + rep * size], np.dtype(dt)


class PSRFITS(object):
    """A memory-mapped fold-mode PSRFITS file: .primary (header dict),
    .subint and .polyco (Table or None)."""

    def __init__(self, filename):
        self.filename = filename
        self._fh = open(filename, "rb")
        size = os.fstat(self._fh.fileno()).st_size
        self._buf = mmap.mmap(self._fh.fileno(), size, access=mmap.ACCESS_READ)
        off = 0
        self.primary, off = _read_header(self._buf, off)
        if not self.primary.get("SIMPLE", False):
            raise ValueError("%s is not a FITS file" % filename)
        off += _data_bytes(self.primary)
        self.subint = self.polyco = None
        while off < size:
            hdr, doff = _read_header(self._buf, off)
            name = str(hdr.get("EXTNAME", "")).strip()
            if hdr.get("XTENSION", "").strip() == "BINTABLE":
                if name == "SUBINT":
                    self.subint = Table(hdr, self._buf, doff)
                elif name == "POLYCO":
                    self.polyco = Table(hdr, self._buf, doff)
            off = doff + _data_bytes(hdr)
        if self.subint is None:
            raise ValueError("%s has no SUBINT table" % filename)
        mode = str(self.primary.get("OBS_MODE", "PSR")).strip()
        if mode not in ("PSR", "CAL", "LEVPSR", "LEVCAL"):
            raise NotImplementedError("OBS_MODE %s: only fold-mode PSRFITS "
                                      "has the fast path" % mode)
        h = self.subint.header
        self.nbin, self.nchan = int(h["NBIN"]), int(h["NCHAN"])
        self.npol = int(h["NPOL"])
        self.nsub = self.subint.nrows
        self.pol_type = str(h.get("POL_TYPE", "AA+BB" if self.npol == 1
                                  else "AABBCRCI")).strip()

    def close(self):
        try:
            self._buf.close()
        except (BufferError, ValueError):
            pass                  # views still alive: the map closes with them
        self._fh.close()

    # -- per sub-int metadata ------------------------------------------------
    def epochs(self):
        """MJD (integer day, fractional day) of every sub-int: STT_IMJD +
        (STT_SMJD + STT_OFFS + OFFS_SUB) / 86400."""
        p = self.primary
        imjd = int(p.get("STT_IMJD", 0))
        sec = float(p.get("STT_SMJD", 0)) + float(p.get("STT_OFFS", 0.0))
        offs = self.subint.column("OFFS_SUB")[:, 0].astype(float) \
            if self.subint.has("OFFS_SUB") else np.zeros(self.nsub)
        tot = sec + offs
        days = np.floor(tot / 86400.0)
        return imjd + days.astype(np.int64), (tot - days * 86400.0) / 86400.0

    def periods(self):
        """Folding period [s] per sub-int: the PERIOD column, else the
        POLYCO table at the sub-int epoch."""
        if self.subint.has("PERIOD"):
            return self.subint.column("PERIOD")[:, 0].astype(float)
        if self.polyco is None or self.polyco.nrows == 0:
            raise ValueError("no PERIOD column and no POLYCO table")
        imjd, frac = self.epochs()
        return np.array([1.0 / polyco_freq(self.polyco, i, f)
                         for i, f in zip(imjd, frac)])

    def freqs(self):
        if self.subint.has("DAT_FREQ"):
            return self.subint.column("DAT_FREQ").astype(float)
        p, h = self.primary, self.subint.header
        bw = float(h.get("CHAN_BW", float(p["OBSBW"]) / self.nchan))
        f0 = float(p["OBSFREQ"]) - (self.nchan - 1) / 2.0 * bw
        return np.tile(f0 + bw * np.arange(self.nchan), (self.nsub, 1))

    def weights(self):
        if self.subint.has("DAT_WTS"):
            return self.subint.column("DAT_WTS").astype(float)
        return np.ones((self.nsub, self.nchan))

    def scales_offsets(self):
        """DAT_SCL, DAT_OFFS as float32 [nsub, npol * nchan] (pol-major)."""
        n = self.npol * self.nchan
        scl = self.subint.column("DAT_SCL").astype(np.float32) \
            if self.subint.has("DAT_SCL") else np.ones((self.nsub, n), np.float32)
        offs = self.subint.column("DAT_OFFS").astype(np.float32) \
            if self.subint.has("DAT_OFFS") else np.zeros((self.nsub, n), np.float32)
        if scl.shape[1] == self.nchan and self.npol > 1:       # per channel only
            scl = np.tile(scl, (1, self.npol))
            offs = np.tile(offs, (1, self.npol))
        return np.ascontiguousarray(scl), np.ascontiguousarray(offs)

    def data_bytes(self):
        """(uint8 view [nsub, npol * nchan * nbin * size], element dtype) of
        the DATA column as stored."""
        return self.subint.column_bytes("DATA")

    def read_data_into(self, nbytes, dst):
        """The first nbytes of every sub-int's DATA cell, read straight from
        the file into dst (a writable uint8 array [nsub, >= nbytes], e.g. a
        pinned buffer) by the native reader (ppf_read_rows: _READ_THREADS
        threads of positioned reads, outside the interpreter lock): no page
        faults on a memory map and no second host copy."""
        from . import _lib
        t = self.subint
        if dst.ndim != 2 or dst.shape[0] < self.nsub or \
                dst.shape[1] < nbytes or dst.strides[1] != 1 or \
                not dst.flags.writeable:
            raise ValueError("read_data_into: dst must be a writable uint8 "
                             "[nsub, >= %d] array with unit column stride"
                             % nbytes)
        rc = _lib.load().ppf_read_rows(
            self._fh.fileno(), t._off + t.columns["DATA"][0], t.rowbytes,
            nbytes, self.nsub, dst.ctypes.data, dst.strides[0],
            _READ_THREADS)
        if rc != 0:
            raise IOError("short read of %s (ppf_read_rows %d)" %
                          (self.filename, rc))


# archive uploads in chunks of this many MiB (env PPF_UPLOAD_CHUNK_MB; 0 =
# one copy): GetTOAs from 16-bit PSRFITS 13.7k vs 13.0k TOAs/s at 16
_UPLOAD_CHUNK = int(os.environ.get("PPF_UPLOAD_CHUNK_MB", "16"))
# threads of the positioned DATA reads (env PPF_READ_THREADS, default 8)
_READ_THREADS = max(1, int(os.environ.get("PPF_READ_THREADS", "8")))


_MASTER = []
_QUEUER = []
# queue the upload and device work on a thread of its own (1) or on the read
# thread after each read (0); env PPF_QUEUE_THREAD
_QUEUE_THREAD = os.environ.get("PPF_QUEUE_THREAD", "1") != "0"


class _Done(object):
    @staticmethod
    def result():
        return None


_DONE = _Done()


def _read_master():
    """The thread that runs one archive's read_data_into at a time (which
    fans out to the native reader threads), so a loader can parse the next file meanwhile."""
    if not _MASTER:
        from concurrent.futures import ThreadPoolExecutor
        _MASTER.append(ThreadPoolExecutor(max_workers=1))
    return _MASTER[0]


def _queuer():
    """The thread that queues each archive's upload and device work once its
    read is done (in read order), so the read of the next archive starts at
    once: the DATA read (≈2.2 ms for 134 MB) and the PCIe upload (≈2.5 ms)
    then overlap instead of alternating with the launch work."""
    if not _QUEUER:
        from concurrent.futures import ThreadPoolExecutor
        _QUEUER.append(ThreadPoolExecutor(max_workers=1))
    return _QUEUER[0]


def polyco_freq(tab, imjd, frac):
    """Spin frequency [Hz] of the TEMPO polyco set nearest the epoch:
    f = REF_F0 + (1/60) sum_i i c_i dt^(i-1), dt in minutes from REF_MJD."""
    ref = tab.column("REF_MJD")[:, 0].astype(float)
    t = imjd + frac
    i = int(np.argmin(np.abs(ref - t)))
    f0 = float(tab.column("REF_F0")[i, 0])
    ncoef = int(tab.column("NCOEF")[i, 0]) if tab.has("NCOEF") else None
    c = tab.column("COEFF")[i].astype(float)
    if ncoef:
        c = c[:ncoef]
    dt = ((imjd - np.floor(ref[i])) + (frac - (ref[i] - np.floor(ref[i])))) \
        * 1440.0
    df = sum(k * c[k] * dt ** (k - 1) for k in range(1, len(c)))
    return f0 + df / 60.0


class _PolycoRows(object):
    """The POLYCO columns polyco_freq reads, copied out of the file map
    (so the map can be closed on the loading thread)."""

    def __init__(self, tab):
        self._c = {k: np.array(tab.column(k)) for k in
                   ("REF_MJD", "REF_F0", "NCOEF", "COEFF") if tab.has(k)}

    def has(self, name):
        return name in self._c

    def column(self, name):
        return self._c[name]


def unpack_host(raw, dtype, scl, offs, npol, nchan, nbin):
    """NumPy restatement of the device unpack (tests): float32 value =
    DATA * DAT_SCL + DAT_OFFS (two float32 roundings, no fused
    multiply-add, as PSRCHIVE's loader computes it), then total intensity:
    npol 1 -> itself, AABBCRCI / AA+BB -> AA + BB, IQUV -> I.
    raw: [nsub, npol * nchan * nbin] file bytes; returns [nsub, nchan, nbin]."""
    nsub = raw.shape[0]
    x = np.ascontiguousarray(raw).view(dtype).reshape(nsub, npol, nchan, nbin)
    x = x.astype(np.float32)
    s = scl.reshape(nsub, npol, nchan, 1).astype(np.float32)
    o = offs.reshape(nsub, npol, nchan, 1).astype(np.float32)
    v = (x * s).astype(np.float32) + o
    return v[:, 0] if npol == 1 else v[:, 0] + v[:, 1]


# ------------------------------------------------------------------ writer --
def _card(key, value, comment=""):
    if isinstance(value, bool):
        v = "%20s" % ("T" if value else "F")
    elif isinstance(value, (int, np.integer)):
        v = "%20d" % value
    elif isinstance(value, (float, np.floating)):
        v = "%20s" % repr(float(value)).upper()
    else:
        v = "'%-8s'" % str(value).replace("'", "''")
    c = "%-8s= %s" % (key, v)
    if comment:
        c += " / " + comment
    return c[:80].ljust(80)


def _header(cards):
    s = "".join(_card(*c) for c in cards) + "END".ljust(80)
    s += " " * (-len(s) % BLOCK)
    return s.encode("ascii")


def write_psrfits(filename, data, scl, offs, freqs, weights, periods,
                  offs_sub, tsubint, stt_imjd=56000, stt_smjd=0, stt_offs=0.0,
                  npol=1, pol_type="AA+BB", telescope="GBT", frontend="Rcvr1_2",
                  backend="GUPPI", source="J1234+5678", dm=0.0, be_delay=0.0,
                  par_ang=None):
    """Write a minimal fold-mode PSRFITS file (primary header + SUBINT
    binary table).  data: int16 [nsub, npol, nchan, nbin]; scl, offs:
    float32 [nsub, npol * nchan]; freqs, weights: [nsub, nchan]; periods,
    offs_sub, tsubint: [nsub]."""
    data = np.asarray(data, dtype=np.int16)
    nsub, npol_, nchan, nbin = data.shape
    assert npol_ == npol
    cols = [("TSUBINT", "1D", None), ("OFFS_SUB", "1D", None),
            ("PERIOD", "1D", None), ("PAR_ANG", "1E", None),
            ("DAT_FREQ", "%dD" % nchan, None), ("DAT_WTS", "%dE" % nchan, None),
            ("DAT_OFFS", "%dE" % (nchan * npol), None),
            ("DAT_SCL", "%dE" % (nchan * npol), None),
            ("DATA", "%dI" % (nbin * nchan * npol), "(%d,%d,%d)" % (nbin, nchan, npol))]
    rowdt = np.dtype([("TSUBINT", ">f8"), ("OFFS_SUB", ">f8"), ("PERIOD", ">f8"),
                      ("PAR_ANG", ">f4"), ("DAT_FREQ", ">f8", (nchan,)),
                      ("DAT_WTS", ">f4", (nchan,)), ("DAT_OFFS", ">f4", (nchan * npol,)),
                      ("DAT_SCL", ">f4", (nchan * npol,)),
                      ("DATA", ">i2", (nbin * nchan * npol,))])
    rows = np.zeros(nsub, dtype=rowdt)
    rows["TSUBINT"] = tsubint
    rows["OFFS_SUB"] = offs_sub
    rows["PERIOD"] = periods
    rows["PAR_ANG"] = 0.0 if par_ang is None else par_ang
    rows["DAT_FREQ"] = freqs
    rows["DAT_WTS"] = weights
    rows["DAT_OFFS"] = offs
    rows["DAT_SCL"] = scl
    rows["DATA"] = data.reshape(nsub, -1)
    obsbw = float(freqs[0, -1] - freqs[0, 0]) * nchan / max(nchan - 1, 1)
    prim = [("SIMPLE", True), ("BITPIX", 8), ("NAXIS", 0), ("EXTEND", True),
            ("HDRVER", "6.1"), ("FITSTYPE", "PSRFITS"), ("OBS_MODE", "PSR"),
            ("TELESCOP", telescope), ("FRONTEND", frontend),
            ("BACKEND", backend), ("SRC_NAME", source),
            ("OBSFREQ", float(np.mean(freqs[0]))), ("OBSBW", obsbw),
            ("OBSNCHAN", nchan), ("STT_IMJD", int(stt_imjd)),
            ("STT_SMJD", int(stt_smjd)), ("STT_OFFS", float(stt_offs)),
            ("BE_DELAY", float(be_delay)), ("CHAN_DM", float(dm))]
    ext = [("XTENSION", "BINTABLE"), ("BITPIX", 8), ("NAXIS", 2),
           ("NAXIS1", rowdt.itemsize), ("NAXIS2", nsub), ("PCOUNT", 0),
           ("GCOUNT", 1), ("TFIELDS", len(cols))]
    for i, (name, form, dim) in enumerate(cols, 1):
        ext += [("TTYPE%d" % i, name), ("TFORM%d" % i, form)]
        if dim:
            ext.append(("TDIM%d" % i, dim))
    ext += [("EXTNAME", "SUBINT"), ("INT_TYPE", "TIME"), ("INT_UNIT", "SEC"),
            ("NPOL", npol), ("POL_TYPE", pol_type), ("NBIN", nbin),
            ("NCHAN", nchan), ("CHAN_BW", float(obsbw / nchan)),
            ("DM", float(dm)), ("NSBLK", 1)]
    body = rows.tobytes()
    with open(filename, "wb") as fh:
        fh.write(_header(prim))
        fh.write(_header(ext))
        fh.write(body)
        fh.write(b"\0" * (-len(body) % BLOCK))
    return filename


def quantize(rows, npol=1):
    """int16 DATA + per-profile float32 DAT_SCL / DAT_OFFS of float rows
    [nsub, npol, nchan, nbin], as a backend digitises them: offset = the
    profile's midrange, scale = half-range / 32767."""
    rows = np.asarray(rows, dtype=np.float64)
    nsub, npol_, nchan, nbin = rows.shape
    lo, hi = rows.min(axis=-1), rows.max(axis=-1)
    offs = ((lo + hi) / 2).astype(np.float32)
    scl = np.maximum((hi - lo) / 2 / 32767.0, 1e-30).astype(np.float32)
    q = np.clip(np.rint((rows - offs[..., None]) / scl[..., None]), -32768,
                32767).astype(np.int16)
    return q, scl.reshape(nsub, npol_ * nchan), offs.reshape(nsub, npol_ * nchan)


# ------------------------------------------------------------- load_data --
def _telescope_code(telescope):
    """pplib.py:2773-2777: the TEMPO2 short code of the telescope
    ($TEMPO2/observatory/observatories.dat when present), else its name."""
    path = os.path.join(os.environ.get("TEMPO2", ""), "observatory",
                        "observatories.dat")
    if os.environ.get("TEMPO2") and os.path.isfile(path):
        with open(path) as fh:
            for ln in fh:
                w = ln.split()
                if w and not ln.startswith("#") and w[-2].upper() == \
                        telescope.upper():
                    return w[-1]
    return telescope


def _window_snr(prof, frac=0.15):
    """S/N of a profile with the baseline window of the device
    (k_base_window / k_row_stats restated): (on-pulse sum) / (sigma_off
    sqrt(n_on)), the window the circular rint(frac nbin)-bin window of
    smallest sum."""
    prof = np.asarray(prof, dtype=float)
    nbin = prof.size
    W = min(nbin - 1, max(1, int(np.rint(frac * nbin))))
    ext = np.concatenate([prof, prof[:W]])
    cs = np.concatenate([[0.0], np.cumsum(ext)])
    b0 = int(np.argmin(cs[W:W + nbin] - cs[:nbin]))
    win = prof[(b0 + np.arange(W)) % nbin]
    mean, sig = win.mean(), win.std()
    on = np.ones(nbin, bool)
    on[(b0 + np.arange(W)) % nbin] = False
    if sig == 0.0 or not on.any():
        return 0.0, sig
    return float((prof[on] - mean).sum() / (sig * np.sqrt(on.sum()))), sig


class DeviceRows(object):
    """load_data's `subints` on the fast path: the float32 rows live in HBM
    ([nsub, nchan, nbin], `.device_rows`); host code that indexes it or
    takes np.asarray gets [nsub, 1, nchan, nbin] (copied back once)."""

    def __init__(self, rows, event):
        self.device_rows, self.event = rows, event
        self._host = None
        n, c, b = rows.shape
        self.shape = (n, 1, c, b)
        self.dtype = np.float32
        self.ndim = 4

    def _get(self):
        if self._host is None:
            if self.event is not None:
                self.event.synchronize()
            self._host = self.device_rows.cpu().numpy()[:, None]
        return self._host

    def __array__(self, dtype=None, copy=None):
        h = self._get()
        return h if dtype is None else h.astype(dtype)

    def __getitem__(self, idx):
        return self._get()[idx]

    def __len__(self):
        return self.shape[0]


class _Masks(object):
    """load_data's `masks` ([nsub, npol, nchan, nbin] 0/1, pplib.py:2859-2861)
    without materialising nsub nchan nbin doubles per archive (537 MB at
    64 x 512 x 2048): indexing builds only the rows asked for."""

    def __init__(self, weights_norm, nbin):
        self.wn, self.nbin = weights_norm, nbin
        self.shape = (weights_norm.shape[0], 1, weights_norm.shape[1], nbin)
        self.ndim = 4

    def _full(self):
        return np.einsum("ij,k", self.wn, np.ones(self.nbin))[:, None]

    def __array__(self, dtype=None, copy=None):
        a = self._full()
        return a if dtype is None else a.astype(dtype)

    def __getitem__(self, idx):
        if isinstance(idx, tuple) and len(idx) == 2 and \
                np.isscalar(idx[0]) and idx[1] == 0:
            return np.repeat(self.wn[idx[0]][:, None], self.nbin, axis=1)
        return self._full()[idx]


# per loading thread and device: a copy stream and a reusable page-locked
# buffer (get_TOAs runs two load_data calls at once on its loader threads)
_TLS = threading.local()


def load_data(filename, state=None, dedisperse=False, dededisperse=False,
              tscrunch=False, pscrunch=False, fscrunch=False, rm_baseline=True,
              flux_prof=False, refresh_arch=True, return_arch=True, quiet=False,
              dev=None, defer=False, lazy=False):
    """pplib.load_data (pplib.py:2749-2915) for fold-mode PSRFITS without
    PSRCHIVE.  The DATA bytes are read from the file into a page-locked
    buffer and uploaded; the device unpacks them, sums the polarisations
    (total intensity: the only state get_TOAs asks for, pscrunch=True),
    removes the baseline and measures every profile
    (ppf_unpack_psrfits_batch), and get_noise_PS gives noise_stds (the
    reference's use_get_noise = True, pplib.py:74, 2841-2848).  The rows stay
    on the device (`subints.device_rows`); get_TOAs fits them without a
    second upload.

    dedisperse / tscrunch follow load_data's order (pplib.py:2786-2793:
    dedisperse, remove the baseline, tscrunch), on the device: every
    channel rotated by the dispersion delay of the stored DM to the centre
    frequency (OBSFREQ), per sub-int period, with the reference's
    rotate_data constant (ppf_rotate_batch), the baseline then measured and
    removed on the dedispersed rows; tscrunch = the DAT_WTS-weighted mean of
    the sub-ints per channel (ppf_align_accum with zero phases; PSRCHIVE's
    weighted Profile average), its weight the summed weights, its epoch the
    middle of the span, its period the predictor's (POLYCO) there or the
    duration-weighted mean PERIOD.  What PSRCHIVE itself would give (its
    dispersion constant, epoch and period conventions) is unpinned here:
    PSRCHIVE is absent and the reference holds no PSRFITS fixture.  A file
    whose data are already dedispersed is not recognised (dmc = 0 on load);
    dededisperse is a no-op.  fscrunch and other polarisation states raise
    NotImplementedError.

    defer=True returns a _Pending whose finish() gives the DataBunch: the
    read is done and the device work queued, but nothing waits for the
    device (get_TOAs' loader thread reads the next archive meanwhile).
    lazy=True (with defer) returns as soon as the file is parsed and its
    DATA read has started on the read thread, which queues the upload and
    device work itself when the read completes (queue() / finish() wait for
    that); without it load_data returns once they are queued."""
    if fscrunch:
        raise NotImplementedError("load_data(fscrunch) needs PSRCHIVE; the "
                                  "PSRFITS fast path keeps every channel")
    if state not in (None, "Intensity"):
        raise NotImplementedError("state=%r needs PSRCHIVE" % state)
    pend = _Pending(filename, pscrunch, state, rm_baseline, quiet, dev,
                    dedisperse=bool(dedisperse), tscrunch=bool(tscrunch))
    if not (defer and lazy):
        pend.queue()
    return pend if defer else pend.finish()


# page-locked DATA buffers per device, used in turn: a buffer is refilled
# only once the upload that read it has completed (its event)
_PINNED = {}
_PINNED_LOCK = threading.Lock()
# page-locked DATA buffers per device (env PPF_PINNED_SLOTS, default 4): a
# read may run this many archives minus one ahead of the oldest upload.
# Archives so large that the slots would pin more than PPF_PINNED_MAX_MB
# (default 4096) rotate through fewer of them (at least two).
_PIN_SLOTS = max(2, int(os.environ.get("PPF_PINNED_SLOTS", "4")))
_PIN_BUDGET = int(os.environ.get("PPF_PINNED_MAX_MB", "4096")) << 20


class _UploadTicket(object):
    """The last user of a pinned slot: synchronize() returns once that
    load has queued its upload (queue()) and the upload has completed."""

    def __init__(self):
        self._done = threading.Event()
        self.ev = None

    def set(self, ev):
        self.ev = ev
        self._done.set()

    def synchronize(self):
        self._done.wait()
        if self.ev is not None:
            self.ev.synchronize()


def _pinned_buffer(dev, nbytes):
    import torch
    with _PINNED_LOCK:
        pool = _PINNED.setdefault(dev.index, dict(
            slots=[[None, None] for _ in range(_PIN_SLOTS)], next=0))
        n = max(2, min(_PIN_SLOTS, _PIN_BUDGET // max(nbytes, 1)))
        i = pool["next"] % n
        pool["next"] = i + 1
        slot = pool["slots"][i]
    buf, ev = slot
    if ev is not None:
        ev.synchronize()
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, pin_memory=True)
        slot[0] = buf
    return buf, slot


# page-locked buffers for the statistics download (stats, total profiles,
# noise), taken by a load and given back once finish() has copied them out
_PACKED = []


def _packed_take(n):
    import torch
    with _PINNED_LOCK:
        for i, b in enumerate(_PACKED):
            if b.numel() >= n:
                return _PACKED.pop(i)[:n]
    return torch.empty(max(n, 1 << 16), dtype=torch.float64,
                       pin_memory=True)[:n]


def _packed_give(buf):
    base = buf._base if buf._base is not None else buf
    with _PINNED_LOCK:
        if len(_PACKED) < 8:
            _PACKED.append(base)


class _Pending(object):
    """load_data's two halves: __init__ parses the file, reads the DATA
    bytes into a page-locked buffer and queues the upload and the device
    unpack / baseline / noise on this thread's copy stream; finish() waits
    for the device and builds the DataBunch."""

    def __init__(self, filename, pscrunch, state, rm_baseline, quiet, dev,
                 dedisperse=False, tscrunch=False):
        import torch
        from . import engine
        from .timeline import span
        self.filename, self.quiet = filename, quiet
        self.dedisperse, self.tscrunch = dedisperse, tscrunch
        with span("load.open"):
            f = self.f = PSRFITS(filename)
            nsub, npol, nchan, nbin = f.nsub, f.npol, f.nchan, f.nbin
            if npol > 1 and not (pscrunch or state == "Intensity"):
                raise NotImplementedError("the PSRFITS fast path returns total "
                                          "intensity (pscrunch=True) only")
            pt = f.pol_type.upper()
            if npol == 1 or pt.startswith("IQUV") or pt == "INTEN":
                pol_mode = 0
            elif pt.startswith("AABB") or pt.startswith("AA+BB"):
                pol_mode = 1
            else:
                raise NotImplementedError("POL_TYPE %s" % f.pol_type)
            raw, edt = f.data_bytes()
            elem = {np.dtype(">i2"): 0, np.dtype("u1"): 1,
                    np.dtype(">f4"): 2}.get(edt)
            if elem is None:
                raise NotImplementedError("DATA element type %s" % edt)
            # only the polarisations total intensity needs cross PCIe: DATA
            # is [npol][nchan][nbin] per sub-int, so AA and BB are its first
            # two npol blocks (2 B / sample / pol for 16-bit data)
            nbytes = (2 if pol_mode == 1 else 1) * nchan * nbin * edt.itemsize
            scl, offs = f.scales_offsets()
            self.weights = f.weights()
            dev = engine.device(dev)
            # host metadata that does not wait for the device
            self.imjd, self.frac = f.epochs()
            self.Ps = f.periods()
            self.freqs = f.freqs()
        # the scales, offsets and weights travel with the DATA bytes: one
        # page-locked buffer holds [DATA rows | DAT_SCL | DAT_OFFS | weights]
        # (float32, 256-B aligned), so the small columns cost no separate
        # pageable copies
        nraw = -(-nsub * nbytes // 256) * 256
        nsc = nsub * npol * nchan
        naux = 4 * (2 * nsc + nsub * nchan)
        with torch.cuda.device(dev):
            buf, slot = _pinned_buffer(dev, nraw + naux)
            # the next user of this slot waits for this load's upload; until
            # the read is submitted, any failure here releases the slot (a
            # ticket that is never set would block that next load for ever)
            self._ticket = slot[1] = _UploadTicket()
        try:
            with torch.cuda.device(dev):
                host = buf[:nsub * nbytes].view(nsub, nbytes)
                aux = buf[nraw:nraw + naux].view(torch.float32)
                a = aux.numpy()
                a[:nsc] = scl.reshape(-1)
                a[nsc:2 * nsc] = offs.reshape(-1)
                a[2 * nsc:] = self.weights.reshape(-1)
            # the rest of the metadata while the file is open
            self.tsub = f.subint.column("TSUBINT")[:, 0].astype(float) \
                if f.subint.has("TSUBINT") else np.zeros(nsub)
            self.par = f.subint.column("PAR_ANG")[:, 0].astype(float) \
                if f.subint.has("PAR_ANG") else np.zeros(nsub)
            self.pred = _PolycoRows(f.polyco) if (
                tscrunch and f.polyco is not None and f.polyco.nrows) else None
            del raw
            self._q = dict(dev=dev, buf=buf, slot=slot, host=host, aux=aux,
                           nraw=nraw, naux=naux, nsc=nsc, nbytes=nbytes,
                           elem=elem, pol_mode=pol_mode,
                           rm_baseline=rm_baseline)
            self._qlock = threading.Lock()
            self._queued = False
            # the DATA read runs on the reader threads from here, and the
            # upload and device work are queued as soon as it completes (on
            # the queueing thread, in read order); queue() / finish() wait
            # for that
            self._rfut = _read_master().submit(self._read_then_queue, nbytes,
                                               host.numpy())
        except BaseException:
            self._ticket.set(None)
            raise
        self._m = self._meta()

    def _read_then_queue(self, nbytes, dst):
        from .timeline import span
        try:
            with span("load.data"):
                self.f.read_data_into(nbytes, dst)
        except BaseException:
            self._ticket.set(None)
            raise
        if not _QUEUE_THREAD:
            self._queue_now()
            return _DONE
        return _queuer().submit(self._queue_now)

    def queue(self):
        """Return once the DATA read is done and the upload, the device
        unpack, baseline, statistics and noise and the statistics download
        are queued (by the queueing thread, on its copy stream)."""
        self._rfut.result().result()

    def _queue_now(self):
        import torch
        from . import engine
        from .timeline import span
        with self._qlock:
            if self._queued:
                return
            self._queued = True
            try:
                self._queue(torch, engine, span)
            finally:
                if not self._ticket._done.is_set():
                    self._ticket.set(None)

    def _queue(self, torch, engine, span):
        q, f = self._q, self.f
        nsub, npol, nchan, nbin = f.nsub, f.npol, f.nchan, f.nbin
        dev, slot, host, aux = q["dev"], q["slot"], q["host"], q["aux"]
        nraw, naux, nsc, nbytes = q["nraw"], q["naux"], q["nsc"], q["nbytes"]
        elem, pol_mode, rm_baseline = q["elem"], q["pol_mode"], \
            q["rm_baseline"]
        dedisperse, tscrunch = self.dedisperse, self.tscrunch
        if not hasattr(_TLS, "streams"):
            _TLS.streams = {}
        with torch.cuda.device(dev):
            # two streams: the uploads queue back to back on the first (the
            # copy engine never waits for an archive's unpack / noise
            # kernels), the device work of each archive on the second after
            # its upload's event
            sts = _TLS.streams.get(dev.index)
            if sts is None:
                sts = _TLS.streams[dev.index] = (torch.cuda.Stream(dev),
                                                 torch.cuda.Stream(dev))
            st_up, st = sts
            with span("load.queue"):
                dbuf = torch.empty(nraw + naux, dtype=torch.uint8, device=dev)
                raw_d = dbuf[:nsub * nbytes].view(nsub, nbytes)
                aux_d = dbuf[nraw:nraw + naux].view(torch.float32)
                with torch.cuda.stream(st_up):
                    aux_d.copy_(aux, non_blocking=True)
                    # in row chunks (PPF_UPLOAD_CHUNK_MB):
                    # a small copy queued meanwhile on another stream (the
                    # fit worker's inputs) need not wait for the whole archive
                    step = max(1, (_UPLOAD_CHUNK << 20) // max(nbytes, 1)) \
                        if _UPLOAD_CHUNK > 0 else nsub
                    for r0 in range(0, nsub, step):
                        raw_d[r0:r0 + step].copy_(host[r0:r0 + step],
                                                  non_blocking=True)
                    up = torch.cuda.Event()
                    up.record(st_up)
                self._ticket.set(up)                # the buffer is free after it
                with torch.cuda.stream(st):
                    st.wait_event(up)
                    # with dedisperse the baseline is removed after the
                    # rotation (pplib.py:2786-2791)
                    out = engine.unpack_psrfits(
                        raw_d, elem, npol, nchan, nbin, aux_d[:nsc],
                        aux_d[nsc:2 * nsc], wts=aux_d[2 * nsc:],
                        pol_mode=pol_mode,
                        rm_baseline=rm_baseline and not dedisperse, dev=dev)
                    if dedisperse or tscrunch:
                        out = self._transform(out, aux_d[2 * nsc:],
                                              rm_baseline, f, dev)
                    noise = engine.noise_rows(out["rows"], dev=dev)
                    # one download: stats [nsub, nchan, 3], total [nsub,
                    # nbin], noise [nsub, nchan] (all float64)
                    packed = torch.cat([out["stats"].reshape(-1),
                                        out["total"].reshape(-1),
                                        noise.reshape(-1)])
                    self.packed_h = _packed_take(packed.numel())
                    self.packed_h.copy_(packed, non_blocking=True)
                    self.ev = torch.cuda.Event()
                    self.ev.record(st)
            self.rows = out["rows"]
            self._keep = (dbuf, packed)
        self._q = None
        # the unmap (milliseconds for a large file) on this thread too
        with span("load.close"):
            f.close()

    def _tscrunched_epoch(self):
        """(imjd [1], frac [1], P [1]) of the tscrunched integration: the
        middle of [first start, last end] (sub-int epochs are centres), the
        period from the POLYCO predictor at it when the file has one, else
        the duration-weighted mean PERIOD."""
        imjd, frac, dur = self.imjd, self.frac, self.tsub
        rel = (imjd - imjd[0]) + frac
        half = dur / 2.0 / 86400.0
        mid = 0.5 * ((rel - half).min() + (rel + half).max())
        day = np.floor(mid)
        i1, f1 = np.array([imjd[0] + int(day)]), np.array([mid - day])
        if self.pred is not None:
            P = np.array([1.0 / polyco_freq(self.pred, int(i1[0]),
                                            float(f1[0]))])
        else:
            w = dur if dur.sum() > 0 else np.ones_like(dur)
            P = np.array([float(np.sum(self.Ps * w) / np.sum(w))])
        return i1, f1, P

    def _transform(self, out, wts, rm_baseline, f, dev):
        """Dedispersion and / or tscrunch of the unpacked rows (on the copy
        stream), then the statistics pass over the result (the native
        float32 rows through ppf_unpack_psrfits_batch, elem 3)."""
        import torch
        from . import engine, pplib
        nsub, nchan, nbin = f.nsub, f.nchan, f.nbin
        rows = out["rows"]
        ones = torch.ones((nsub, nchan), dtype=torch.float32, device=dev)
        zeros = torch.zeros((nsub, nchan), dtype=torch.float32, device=dev)

        def stats(rows, w, rm):
            n = rows.shape[0]
            return engine.unpack_psrfits(
                rows.reshape(n, nchan * nbin).view(torch.uint8), 3, 1, nchan,
                nbin, ones[:n], zeros[:n], wts=w, pol_mode=0, rm_baseline=rm,
                dev=dev)
        if self.dedisperse:
            # rotate_data(rows, 0, DM, Ps, freqs, nu0) (pplib.py:2427-2515):
            # the phases as it forms them
            p, h = f.primary, f.subint.header
            DM = float(h.get("DM", p.get("CHAN_DM", 0.0)))
            nu0 = float(p.get("OBSFREQ", self.freqs.mean()))
            D = pplib.Dconst * DM / (np.ones(nsub) * self.Ps)
            ph = D[:, None] * (self.freqs ** -2.0 - nu0 ** -2.0)
            rows = engine.rotate_rows(rows, ph, dev=dev).float()
            out = stats(rows, wts, rm_baseline)
            rows = out["rows"]
        if self.tscrunch:
            acc = torch.zeros((nchan, nbin), dtype=torch.float64, device=dev)
            wsum = torch.zeros(nchan, dtype=torch.float64, device=dev)
            engine.align_accum(rows, torch.zeros((nsub, nchan),
                                                 dtype=torch.float64,
                                                 device=dev),
                               wts.reshape(nsub, nchan).double(), acc, wsum,
                               dev=dev)
            mean = acc / torch.where(wsum > 0, wsum,
                                     torch.ones_like(wsum))[:, None]
            out = stats(mean.float()[None].contiguous(),
                        wsum.float()[None].contiguous(), False)
        return out

    def finish(self):
        from .timeline import span
        with span("load.read"):
            self.queue()                    # read and queued (or raised)
        with span("load.wait"):
            self.ev.synchronize()
        self._keep = None
        with span("load.meta"):
            data = self._bunch()
        _packed_give(self.packed_h)
        self.packed_h = None
        return data

    def _meta(self):
        """The DataBunch fields that need only the file (built on the loading
        thread while the DATA read runs)."""
        from . import pplib
        f, filename, weights = self.f, self.filename, self.weights
        nsub, nchan, nbin = f.nsub, f.nchan, f.nbin
        prof_norm = max(1.0, float(np.count_nonzero(weights)))
        imjd, frac, Ps, freqs = self.imjd, self.frac, self.Ps, self.freqs
        tsub, par = self.tsub, self.par
        doppler = np.ones(nsub)
        if self.tscrunch:
            # one integration: summed weights, the middle of the span, the
            # period there, the summed duration
            imjd, frac, Ps = self._tscrunched_epoch()
            weights = weights.sum(axis=0)[None]
            freqs = freqs[:1]
            par = np.array([par.mean()])
            doppler = np.ones(1)
            nsub = 1
        p, h = f.primary, f.subint.header
        epochs = [pplib.MJD(int(i), float(x)) for i, x in zip(imjd, frac)]
        weights_norm = np.where(weights == 0.0, 0.0, 1.0)
        ok_isubs = np.compress(weights_norm.mean(axis=1), list(range(nsub)))
        chans = np.arange(nchan)
        okc = weights_norm != 0.0
        if okc.all():
            ok_ichans = [chans] * nsub
        else:
            ok_ichans = [chans[okc[isub]] for isub in range(nsub)]
        telescope = str(p.get("TELESCOP", "")).strip()
        return dict(
            _nsub=nsub, _prof_norm=prof_norm,
            arch=None, backend=str(p.get("BACKEND", "")).strip(),
            backend_delay=float(p.get("BE_DELAY", 0.0)),
            bw=float(p.get("OBSBW", 0.0)), doppler_factors=doppler,
            doppler_known=False, DM=float(h.get("DM", p.get("CHAN_DM", 0.0))),
            dmc=int(self.dedisperse), epochs=epochs, filename=filename,
            flux_prof=np.array([]),
            freqs=freqs, frontend=str(p.get("FRONTEND", "")).strip(),
            integration_length=float(tsub.sum()),
            masks=_Masks(weights_norm, nbin), nbin=nbin, nchan=nchan,
            npol=1, nsub=nsub,
            nu0=float(p.get("OBSFREQ", self.freqs.mean())),
            ok_ichans=ok_ichans, ok_isubs=ok_isubs, parallactic_angles=par,
            phases=pplib.get_bin_centers(nbin), Ps=Ps,
            source=str(p.get("SRC_NAME", "")).strip(), state="Intensity",
            subtimes=[float(tsub.sum())] if self.tscrunch else list(tsub),
            telescope=telescope, telescope_code=_telescope_code(telescope),
            weights=weights)

    def _bunch(self):
        from . import pplib
        m = dict(self._m)
        nsub, prof_norm = m.pop("_nsub"), m.pop("_prof_norm")
        nchan, nbin = m["nchan"], m["nbin"]
        packed = self.packed_h.numpy()
        n1, n2 = nsub * nchan * 3, nsub * nbin
        stats = packed[:n1].reshape(nsub, nchan, 3)
        total = packed[n1:n1 + n2].reshape(nsub, nbin)
        # (copies: the page-locked buffer goes back to its pool)
        noise = packed[n1 + n2:n1 + n2 + nsub * nchan].reshape(nsub, nchan)
        prof = total.sum(axis=0)
        prof_SNR, prof_noise = _window_snr(prof)
        if not self.quiet:
            print("\nReading data from %s on source %s (PSRFITS fast "
                  "path)..." % (self.filename, m["source"]))
        return pplib.DataBunch(
            noise_stds=noise[:, None, :].copy(), prof=prof / prof_norm,
            prof_noise=prof_noise, prof_SNR=prof_SNR,
            SNRs=stats[:, None, :, 2].copy(),
            subints=DeviceRows(self.rows, self.ev), **m)

"""Drop-in mirror of PulsePortraiture's ``ppzap`` channel flagger.

Two ways to propose channels to zap (reference: /root/reference/ppzap.py):
the noise-median iteration ``get_zap_channels`` (host arithmetic over the
per-channel noise levels that ``load_data`` computes with the device
``get_noise_PS``), and the model-based cut, ``GetTOAs.get_TOAs`` followed by
``GetTOAs.get_channels_to_zap`` (per-channel reduced chi^2 on the GPU,
``ppf_resid_chi2_batch``).  ``print_paz_cmds`` writes the PSRCHIVE ``paz``
commands exactly as the reference does.
"""
import sys

import numpy as np

from . import pptoas
from .pplib import file_is_type, get_noise
from .pptoas import GetTOAs, rm_baseline


def get_zap_channels(data, nstd=3):
    """ppzap.py:23-53: per sub-integration, flag channels whose noise level
    exceeds median + nstd * std of the remaining channels, remove them and
    iterate until none is flagged.  Returns [isub] sorted channel lists."""
    zap_channels = []
    for isub in data.ok_isubs:
        ichans = list(np.copy(data.ok_ichans[isub]))
        zap_ichans = []
        while len(ichans):
            noise_stds = data.noise_stds[isub, 0, ichans]
            median = np.median(noise_stds)
            std = np.std(noise_stds)
            bad = list(np.where(noise_stds > median + nstd * std)[0])
            if not len(bad):
                break
            flagged = np.array(ichans)[bad]
            zap_ichans.extend(list(flagged))
            for ichan in flagged:
                ichans.pop(ichans.index(ichan))
        zap_ichans.sort()
        zap_channels.append(zap_ichans)
    return zap_channels


def print_paz_cmds(datafiles, zap_list, all_subs=False, modify=True,
                   outfile=None, quiet=False):
    """ppzap.py:56-106: ``paz`` commands for zap_list[iarch][isub]; with
    all_subs a channel is zapped in every sub-integration (consecutive
    duplicates dropped); modify=False writes to a '.zap' copy.  outfile
    appends instead of printing."""
    if not len(datafiles) or not len(zap_list):
        if not quiet:
            print("Nothing to zap.")
            return None
    prev_stdout = sys.stdout
    if outfile is not None:
        sys.stdout = open(outfile, "a")
    try:
        for iarch, datafile in enumerate(datafiles):
            count = sum(len(z) for z in zap_list[iarch])
            if count:
                if modify:
                    paz_outfile = datafile
                else:
                    ii = datafile[::-1].find(".")
                    paz_outfile = datafile + ".zap" if ii < 0 else \
                        datafile[:-ii] + "zap"
                    print("paz -e zap %s" % datafile)
            last_line = ""
            for isub, bad_ichans in enumerate(zap_list[iarch]):
                for bad_ichan in bad_ichans:
                    if not all_subs:
                        print("paz -m -I -z %d -w %d %s" % (bad_ichan, isub,
                                                            paz_outfile))
                    else:
                        line = "paz -m -z %d %s" % (bad_ichan, paz_outfile)
                        if line != last_line:
                            print(line)
                        last_line = line
    finally:
        if outfile is not None:
            sys.stdout.close()
        sys.stdout = prev_stdout     # the reference resets to sys.__stdout__
    if outfile is not None and not quiet:
        print("Wrote %s." % outfile)


def main(argv=None):
    """The ppzap.py command line (ppzap.py:109-253), minus --hist (plotting)
    and --norm (portrait normalisation; outside the accelerated path)."""
    from optparse import OptionParser
    parser = OptionParser("Usage: %prog -d <datafile or metafile> [options]")
    parser.add_option("-d", "--datafiles", dest="datafiles")
    parser.add_option("-n", "--num_std", dest="nstd", default=5.0)
    parser.add_option("-N", "--norm", dest="norm", default=None)
    parser.add_option("-m", "--modelfile", dest="modelfile", default=None)
    parser.add_option("-T", "--tscrunch", action="store_true",
                      dest="tscrunch", default=False)
    parser.add_option("-S", "--SNR-threshold", dest="SNR_threshold",
                      default=8.0)
    parser.add_option("-R", "--rchi2-threshold", dest="rchi2_threshold",
                      default=1.3)
    parser.add_option("-o", "--outfile", dest="outfile", default=None)
    parser.add_option("--modify", action="store_true", dest="modify",
                      default=False)
    parser.add_option("--hist", action="store_true", dest="hist",
                      default=False)
    parser.add_option("--quiet", action="store_true", dest="quiet",
                      default=False)
    options, _ = parser.parse_args(argv)
    if options.datafiles is None:
        print("\nppzap.py - Identify bad channels to zap.\n")
        parser.print_help()
        print("")
        return 0
    if options.hist or options.norm is not None:
        raise NotImplementedError("--hist / --norm are outside the "
                                  "accelerated path (SURVEY.md section 2)")
    datafiles = options.datafiles
    tscrunch, quiet = options.tscrunch, options.quiet
    if options.modelfile is not None:
        gt = GetTOAs(datafiles=datafiles, modelfile=options.modelfile,
                     quiet=True)
        gt.get_TOAs(tscrunch=tscrunch, quiet=True)
        gt.get_channels_to_zap(SNR_threshold=float(options.SNR_threshold),
                               rchi2_threshold=float(options.rchi2_threshold),
                               iterate=True, show=False)
        ok_datafiles = list(np.array(gt.datafiles)[gt.ok_idatafiles])
        print_paz_cmds(ok_datafiles, gt.zap_channels, all_subs=tscrunch,
                       modify=options.modify, outfile=options.outfile,
                       quiet=quiet)
        nchan = sum(len(c) for a in gt.channel_red_chi2s[:len(ok_datafiles)]
                    for c in a)
        nzap = sum(len(z) for a in gt.zap_channels[:len(ok_datafiles)]
                   for z in a)
        if not quiet:
            print("ppzap.py found %d channels to zap out of a total %d "
                  "channels fit (=%.2f%%) in %s." % (
                      nzap, nchan, 100 * float(nzap) / nchan, datafiles))
        return 0
    if file_is_type(datafiles, "ASCII"):
        with open(datafiles) as fh:
            all_datafiles = [ln[:-1] for ln in fh.readlines()]
    else:
        all_datafiles = [datafiles]
    nchan, zap_channels = 0, []
    for datafile in all_datafiles:
        try:
            data = pptoas.load_data(
                datafile, dedisperse=False, dededisperse=False,
                tscrunch=tscrunch, pscrunch=True, fscrunch=False,
                rm_baseline=rm_baseline, flux_prof=False, refresh_arch=False,
                return_arch=False, quiet=True)
        except RuntimeError:
            if not quiet:
                print("Cannot load_data(%s).  Skipping it." % datafile)
            continue
        nchan += int(np.array(list(map(len, data.ok_ichans))).sum())
        zap_channels.append(get_zap_channels(data,
                                             nstd=float(options.nstd)))
    print_paz_cmds(all_datafiles, zap_channels, all_subs=tscrunch,
                   modify=options.modify, outfile=options.outfile,
                   quiet=quiet)
    nzap = sum(len(z) for a in zap_channels for z in a)
    if not quiet:
        print("ppzap.py found %d channels to zap out of a total %d channels "
              "(=%.2f%%) in %s." % (nzap, nchan, 100 * float(nzap) / nchan,
                                    datafiles))
    return 0


__all__ = ["get_zap_channels", "print_paz_cmds", "main", "get_noise"]

if __name__ == "__main__":
    sys.exit(main())

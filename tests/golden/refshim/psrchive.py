"""Import-time stand-in for the PSRCHIVE SWIG module (absent in this image).

Only ``MJD`` arithmetic is reachable from the code paths the golden-vector
generator exercises (``epoch + pr.MJD(seconds / 86400)`` in get_TOAs); it is
kept as float days, so golden TOAs record phases, never absolute MJDs.
"""


class MJD(object):
    def __init__(self, *a):
        self.days = float(a[0]) if a else 0.0

    def __add__(self, other):
        if isinstance(other, MJD):
            return MJD(self.days + other.days)
        return MJD(self.days + other / 86400.0)

    def in_days(self):
        return self.days

    def intday(self):
        return int(self.days)

    def fracday(self):
        return self.days - int(self.days)

    def printdays(self, ndigits):
        return ("%%.%df" % ndigits) % self.days

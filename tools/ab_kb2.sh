# round 6: KB = 3 (default now, seeds every 64 harmonics) against KB = 4, after
# the scattering / fit parity tests on the new default
TESTK="c3 or c5 or scat or fullshape or full_matches or chime or pdta" bash tools/ab.sh kb2 "c3 c5" "base lib:varlib/libppfit_kb4.so" 2

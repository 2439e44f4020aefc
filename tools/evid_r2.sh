#!/bin/bash
# Round-2 counter evidence: kernel stats + FETCH/WRITE + SQ/f64 passes for
# the C2 (phase+DM), C3 (full) and C5 (scat) bench shapes.
set -e
bash tools/prof.sh c2 --nsub 2500 --passes 1
bash tools/prof.sh c3 --fit full --nsub 2500
bash tools/prof.sh c5 --fit scat --nchan 16384 --nbin 1024 --nsub 100

#!/bin/bash
# Round-3 final evidence: the full GPU parity suite and every bench line
# (tools/evid_r3.sh), then the rocprofv3 kernel statistics and counter
# passes (tools/prof_r3.sh).  usage: tools/final_r3.sh TAG
set -e
tag=${1:-f}
bash tools/evid_r3.sh $tag tests
bash tools/prof_r3.sh r3$tag

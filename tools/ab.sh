#!/bin/bash
# A/B driver (GPU box, one gpurun call): every named bench config under every
# variant, REPS times, in one call (box-to-box spread is ~10 %, so only
# same-call comparisons count).  A variant is `lib:PATH` (a libppfit build,
# e.g. varlib/libppfit_NAME.so from tools/build_variant.sh), `env:K=V[,K=V]`
# (environment settings) or `base` (the default library and environment).
# Optionally runs a GPU test subset first (TESTK="pytest -k expression",
# TESTK=all: the whole GPU suite).
#   usage: tools/ab.sh TAG "c2 c3 c5 c4 gtps gt nb1000 nb1536" "base lib:... env:..." [REPS]
#   out:   gpurun_out/ab_TAG/{CONFIG}_{VARIANT}_{REP}.json, ab_TAG/status.txt
tag=$1; cfgs=$2; vars=$3; reps=${4:-1}
export TMPDIR=/tmp
out=gpurun_out/ab_$tag
mkdir -p $out
st=$out/status.txt
if [ -n "$TESTK" ]; then
  kx=(); [ "$TESTK" != all ] && kx=(-k "$TESTK")
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "${kx[@]}" > $out/pytest.log 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 $out/pytest.log)" >> $st
  [ $rc -eq 0 ] || exit $rc
fi
args_of() {
  case $1 in
    c2) echo "--cpu-sample 0";;
    c3) echo "--fit full --nsub 10000 --steps 3 --warmup 1 --cpu-sample 0";;
    c5) echo "--fit scat --nchan 16384 --nbin 1024 --nsub 500 --steps 3 --warmup 1 --cpu-sample 0";;
    c4) echo "--fit align --nsub 1000 --nchan 256 --nbin 1024 --steps 50 --warmup 5 --cpu-sample 0";;
    c4n512) echo "--fit align --nsub 1000 --nchan 256 --nbin 512 --steps 50 --warmup 5 --cpu-sample 0";;
    c4n2048) echo "--fit align --nsub 1000 --nchan 256 --nbin 2048 --steps 50 --warmup 5 --cpu-sample 0";;
    gtps) echo "--fit gettoas --psrfits --steps 4 --warmup 1";;
    gt) echo "--fit gettoas --steps 3 --warmup 1";;
    nb1000) echo "--nbin 1000 --nsub 4000 --steps 3 --warmup 1 --cpu-sample 0";;
    nb1536) echo "--nbin 1536 --nsub 4000 --steps 3 --warmup 1 --cpu-sample 0";;
    nb1022) echo "--nbin 1022 --nsub 4000 --steps 3 --warmup 1 --cpu-sample 0";;
    nb1023) echo "--nbin 1023 --nsub 4000 --steps 3 --warmup 1 --cpu-sample 0";;
    *) echo "BAD";;
  esac
}
for rep in $(seq 1 $reps); do
  for c in $cfgs; do
    a=$(args_of $c)
    [ "$a" = BAD ] && { echo "unknown config $c" >> $st; exit 2; }
    for v in $vars; do
      envs=(); lib=""
      case $v in
        base) ;;
        lib:*) lib=${v#lib:};;
        env:*) IFS=, read -ra envs <<< "${v#env:}";;
      esac
      name=$(echo "$v" | tr '/:=,.' '_____')
      f=$out/${c}_${name}_$rep.json
      env "${envs[@]}" ${lib:+PPFIT_LIB=$lib} timeout -k 10 300 python bench.py $a > $f 2> ${f%.json}.err
      rc=$?
      echo "$c $v $rep rc=$rc $(python tools/show.py $f 2>/dev/null | head -1)" >> $st
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
echo end >> $st

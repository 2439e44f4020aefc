#!/bin/bash
# Build an experimental libppfit variant: tools/build_variant.sh NAME "-DMACRO=1 ..."
# -> varlib/libppfit_NAME.so (select with PPFIT_LIB=...)
set -e
name=$1; shift
flags="$*"
root=$(cd $(dirname $0)/.. && pwd)
od=$root/varlib/tmp_$name
mkdir -p $od
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-pass-failed -ffp-contract=fast -munsafe-fp-atomics $flags"
C=$root/pulseportraiture_amd/csrc
$H -c $C/ppf_kernels.hip -o $od/k.o &
$H -c $C/ppf_xspec.hip -o $od/x.o &
$H -c $C/ppf_longfft.hip -o $od/l.o &
$H -c $C/ppf_solve.hip -o $od/s.o &
$H -c $C/ppf_psrfits.hip -o $od/p.o &
$H -x hip -c $C/ppf_api.cpp -o $od/a.o &
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -Wall -pthread -c $C/ppf_io.cpp -o $od/i.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -pthread -o $root/varlib/libppfit_$name.so $od/k.o $od/l.o $od/x.o $od/s.o $od/p.o $od/a.o $od/i.o
rm -rf $od
echo built varlib/libppfit_$name.so

#!/bin/bash
# Build experiment variants of libsrbd_hip.so: NAME:"-DFLAGS ..." pairs -> quadruped-pympc-tamols_amd/variants/lib_NAME.so
# (measurement only; scripts/vrun.sh / variant_probe.py load each through SRBD_LIB_PATH).  FILES (env, default
# "srbd_rollout_thread") lists the translation units rebuilt with the flags; the rest come from build/.
set -e
cd "$(dirname "$0")/../quadruped-pympc-tamols_amd"
make -s -j8 >/dev/null
mkdir -p variants
FILES=${FILES:-srbd_rollout_thread}
for spec in "$@"; do
    name=${spec%%:*}; flags=${spec#*:}
    d=build/var_$name; rm -rf $d; mkdir -p $d
    for o in build/*.o; do cp $o $d/; done
    for f in $FILES; do
        extra=""; [ "$f" = srbd_rollout_thread ] && extra=-fno-slp-vectorize
        /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function $extra $flags -c csrc/$f.hip -o $d/$f.o &
    done
    wait
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o variants/lib_$name.so $d/*.o -ldl
    echo "built variants/lib_$name.so ($flags)"
done

#!/bin/bash
# Builds an A/B variant of libgsv.so with extra -D flags (sources in $VSRCS, default ecrecover notary)
# into variants/<name>/ (git-ignored,
# shipped to the GPU box); select it at run time with GSV_LIB_PATH=variants/<name>/libgsv.so.
set -e
name=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/variants/$name
cd $R/geth-sharding_amd/csrc
make -s -j8 >/dev/null
pids=""
VSRCS=${VSRCS:-ecrecover notary}
for f in $VSRCS; do
    /opt/rocm/bin/hipcc "$@" -O3 -std=c++17 -fPIC --offload-arch=gfx950 -c $f.hip -o $R/variants/$name/$f.o 2>&1 | grep -v hip-link || true &
done
wait
for f in gsv_api keccak ecrecover chunk_root tx_host bn256 notary collation; do
    case " $VSRCS " in *" $f "*) ;; *) cp build/$f.o $R/variants/$name/ ;; esac
done
/opt/rocm/bin/hipcc -fPIC --offload-arch=gfx950 -shared -o $R/variants/$name/libgsv.so $R/variants/$name/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $R/variants/$name/libgsv.so

#!/bin/bash
# Build an A/B variant of the Python extension with extra compile flags for the Equihash solver.
# Usage: bash tools/build_variant.sh NAME [-DFLAG=V ...]  ->  ab/NAME/_bcpnative*.so
# (run `make pyext` first; only csrc/kernels/equihash_solver.hip, or $SRC, is recompiled)
set -e
cd "$(dirname "$0")/.."
NAME=$1
shift
EXT=$(python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
D=build/var/$NAME
mkdir -p "$D" ab/"$NAME"
/opt/rocm/bin/hipcc -std=c++17 -O2 -fPIC --offload-arch=gfx950 -Icsrc -munsafe-fp-atomics -Wno-unused-result \
    -Wno-unused-variable -Wno-pass-failed "$@" -c "${SRC:-csrc/kernels/equihash_solver.hip}" -o "$D/equihash_solver.o"
cp build/libbcpcore.a "$D/libbcpcore.a"
ar r "$D/libbcpcore.a" "$D/equihash_solver.o"
g++ -shared -o ab/"$NAME"/_bcpnative"$EXT" build/obj/python/*.o -Wl,--whole-archive "$D/libbcpcore.a" \
    -Wl,--no-whole-archive -L/opt/rocm/lib -lamdhip64 -lcrypto -pthread -ldl -Wl,-rpath,/opt/rocm/lib
echo "built ab/$NAME/_bcpnative$EXT"

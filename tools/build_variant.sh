#!/bin/bash
# Build an A/B variant of the Python extension with extra compile flags for one kernel file
# (default the Equihash solver; OBJ=secp256k1 SRC=path.hip for another one).
# Usage: [OBJ=name] [SRC=file.hip] bash tools/build_variant.sh NAME [-DFLAG=V ...]  ->  ab/NAME/_bcpnative*.so
# (run `make pyext` first; only csrc/kernels/equihash_solver.hip, or $SRC, is recompiled)
set -e
cd "$(dirname "$0")/.."
NAME=$1
shift
EXT=$(python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
D=build/var/$NAME
mkdir -p "$D" ab/"$NAME"
# the Makefile's per-file flags of the solver (HIPFLAGS_equihash_solver) unless EH_FLAGS overrides them
[ "${OBJ:-equihash_solver}" = equihash_solver ] && DEF=${EH_FLAGS-"-mllvm -amdgpu-sched-strategy=max-ilp -mllvm -amdgpu-use-amdgpu-trackers=1 -mllvm -amdgpu-atomic-optimizer-strategy=None"} || DEF=""
/opt/rocm/bin/hipcc -std=c++17 -O2 -fPIC --offload-arch=gfx950 -Icsrc -munsafe-fp-atomics -Wno-unused-result \
    -Wno-unused-variable -Wno-pass-failed $DEF "$@" -c "${SRC:-csrc/kernels/${OBJ:-equihash_solver}.hip}" -o "$D/${OBJ:-equihash_solver}.o"
cp build/libbcpcore.a "$D/libbcpcore.a"
# replace the kernel's member (the LAST one of that name: csrc/secp256k1/secp256k1.o, the CPU library,
# shares the kernel object's basename and comes first in the archive)
M=${OBJ:-equihash_solver}.o
CNT=$(ar t "$D/libbcpcore.a" | grep -cx "$M")
ar dN "$CNT" "$D/libbcpcore.a" "$M"
cp "$D/$M" "$D/k_$M"
ar r "$D/libbcpcore.a" "$D/k_$M"
g++ -shared -o ab/"$NAME"/_bcpnative"$EXT" build/obj/python/*.o -Wl,--whole-archive "$D/libbcpcore.a" \
    -Wl,--no-whole-archive -L/opt/rocm/lib -lamdhip64 -lcrypto -pthread -ldl -Wl,-rpath,/opt/rocm/lib
echo "built ab/$NAME/_bcpnative$EXT"

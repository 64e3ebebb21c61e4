set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tl1
mkdir -p $O
export TMPDIR=/tmp
EXT=_bcpnative.cpython-310-x86_64-linux-gnu.so
for b in $(ls ab); do
  (cd /tmp && BCP_NATIVE_PATH=$R/ab/$b/$EXT timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$O/$b" -o run -- \
    python3 "$R/bench.py" --steps 6 --warmup 2 > "$O/$b.log" 2>&1)
  python3 tools/eh_timeline.py "$O/$b" 60 > "$O/$b.txt"
  head -n 16 "$O/$b.txt"
done
echo DONE

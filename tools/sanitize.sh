#!/bin/bash
# Host sanitizer runs of the node (reference --enable-tsan / --enable-asan, configure.ac:195-275).
#   tools/sanitize.sh tsan   -> ThreadSanitizer: unit suites + every functional test vs bin/tsan/bcpd
#   tools/sanitize.sh asan   -> AddressSanitizer + UBSan: the same against bin/asan/bcpd
# Reports land in $OUT (one file per process); the script fails if any were written.
# GPU code is never sanitized (the gfx950 kernel objects are linked as they are).
set -u
cd "$(dirname "$0")/.."
MODE=${1:-tsan}
OUT=${2:-/tmp/bcp_sanitize_$MODE}
rm -rf "$OUT" && mkdir -p "$OUT"
case "$MODE" in
  tsan) make -j8 tsan > "$OUT/build.log" 2>&1 || { echo "build failed"; exit 2; }
        export TSAN_OPTIONS="log_path=$OUT/report halt_on_error=0 second_deadlock_stack=1" ;;
  asan) make -j8 asan-node > "$OUT/build.log" 2>&1 || { echo "build failed"; exit 2; }
        export ASAN_OPTIONS="log_path=$OUT/report detect_leaks=0"
        export UBSAN_OPTIONS="log_path=$OUT/report print_stacktrace=1" ;;
  *) echo "usage: $0 tsan|asan [outdir]"; exit 2 ;;
esac
(cd "$OUT" && "$OLDPWD/bin/$MODE/test_bcp") > "$OUT/unit.log" 2>&1
unit=$?
BCP_BCPD="$PWD/bin/$MODE/bcpd" python -m pytest -q tests/ -m "functional and not gpu" -n 4 -p no:cacheprovider \
  > "$OUT/functional.log" 2>&1
func=$?
reports=$(ls "$OUT"/report.* 2>/dev/null | wc -l)
echo "$MODE: unit rc=$unit ($(tail -1 "$OUT/unit.log")), functional rc=$func ($(tail -1 "$OUT/functional.log")), reports=$reports"
[ "$unit" = 0 ] && [ "$func" = 0 ] && [ "$reports" = 0 ]

set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abbatch
for cfg in "32 2" "64 2" "32 3" "48 2" "32 2"; do
  set -- $cfg
  timeout -k 10 240 python bench.py --steps 12 --warmup 3 --batch $1 --solvers $2 > gpurun_out/abbatch/b$1_s$2.json 2>gpurun_out/abbatch/b$1_s$2.err
  echo "batch $1 solvers $2: $(python3 -c "import json;d=json.load(open('gpurun_out/abbatch/b$1_s$2.json'));print(d['value'], d['ms_per_step'], d['config']['solutions_per_nonce'])")"
done

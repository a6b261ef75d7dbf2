# Alternating timing of library builds tools/bin/lib_<name>.so on config 3 (one 16-bit
# adder, the latency form): bash tools/gpu_ab_adder.sh TAG ROUNDS name1 name2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; R=$2; shift 2
for r in $(seq 1 $R); do
  for v in "$@"; do
    TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$PWD/tools/bin/lib_$v.so timeout -k 10 200 python bench.py --workload adder --batch 1 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_$v$r.json 2> gpurun_out/${T}_$v$r.err || { echo "$v failed"; tail -5 gpurun_out/${T}_$v$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d.get('ms_per_step'), d.get('decrypt_check', d.get('correct')))" gpurun_out/${T}_$v$r.json "$v r$r"
  done
done

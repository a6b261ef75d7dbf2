# N>1 rehearsals on one GPU: 2 gloo ranks sharing the card, and the single-process context with the device twice
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/reh_gloo2.json 2> gpurun_out/reh.err || { echo "gloo2 failed"; tail -20 gpurun_out/reh.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('gloo 2 ranks', d['n_gpus'], d['value'], d['ms_per_step'], d.get('decrypt_check'))" gpurun_out/reh_gloo2.json
timeout -k 10 300 python bench.py --single-process --gpus 2 --devices 0,0 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/reh_sp2.json 2> gpurun_out/reh.err || { echo "sp2 failed"; tail -20 gpurun_out/reh.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('single-process 2 shards', d['n_gpus'], d['value'], d['ms_per_step'], d.get('decrypt_check'))" gpurun_out/reh_sp2.json

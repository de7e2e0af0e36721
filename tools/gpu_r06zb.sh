# round 6, call zb: smoke() and the distributed bench path on the final tree (RCCL at one rank, plain and under
# torch.distributed.run)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06zb_smoke.log 2>&1 || { tail -20 gpurun_out/r06zb_smoke.log; exit 1; }
tail -3 gpurun_out/r06zb_smoke.log
timeout -k 10 300 python bench.py --rccl --no-legs --no-cpu-baseline --steps 40 --warmup 5 > gpurun_out/r06zb_rccl.json 2> gpurun_out/r06zb_rccl.err || { tail -20 gpurun_out/r06zb_rccl.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 40 --warmup 5 --no-legs --no-cpu-baseline > gpurun_out/r06zb_torchrun.json 2> gpurun_out/r06zb_torchrun.err || { tail -20 gpurun_out/r06zb_torchrun.err; exit 1; }
python -c "
import json
for f in ('gpurun_out/r06zb_rccl.json', 'gpurun_out/r06zb_torchrun.json'):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['config'].get('parallelism'), d.get('n_gpus'))
"

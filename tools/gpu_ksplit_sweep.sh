for ks in 0 2 3 4 8; do
  AVSE_GEMM_KSPLIT=$ks timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/ks_$ks.json 2>/dev/null || exit $?
  python -c "import json; d=json.load(open('gpurun_out/ks_$ks.json')); s=d['breakdown']['stage_ms']; print($ks, d['ms_per_step'], s['v_conv6'], s['enc_dense'], s['dec_dense1'], s['dec_dense2'])"
done

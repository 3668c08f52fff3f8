# Wave census of the C3 pipeline in N separate processes (the producer's placement varies
# from process to process): gpurun_out/census_<i>.{json,npz}, one line of producer spans each
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in $(seq ${N:-8}); do
  timeout -k 10 120 python -u tools/census.py --steps 6 --warmup 6 --out gpurun_out/census_$i.npz > gpurun_out/census_$i.json 2> gpurun_out/census_$i.err || { tail -5 gpurun_out/census_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/census_$i.json'))
print($i, [round(v['span_us']) for k, v in d['kernels'].items() if 'rng_parser' in k])"
done

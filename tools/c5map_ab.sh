cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in 0 1; do
LSLAM_RNG_SELF=$v timeout -k 10 300 python -u tools/c5bench.py --scans 4096 --reps 2 > gpurun_out/c5_$v.json 2> gpurun_out/c5_$v.err || { tail -5 gpurun_out/c5_$v.err; exit 1; }
echo "SELF=$v"; cat gpurun_out/c5_$v.json
LSLAM_RNG_SELF=$v timeout -k 10 300 python -u tools/mapbench.py > gpurun_out/map_$v.json 2> gpurun_out/map_$v.err || { tail -5 gpurun_out/map_$v.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/map_$v.json')); print('map', d['value'], d['ms_per_step'])"
done

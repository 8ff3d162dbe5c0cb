set -eu -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep1
for n in 1 4 16 64; do
  timeout -k 10 120 python -u bench.py --png-only --no-cpu-baseline --images $n --distinct 1 > gpurun_out/sweep1/n$n.json 2> gpurun_out/sweep1/n$n.err
  python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], r['roofline']['kernel_ms_per_launch'])" gpurun_out/sweep1/n$n.json $n
done
for n in 1 64; do
  ZPX_PNG_PAIR=0 timeout -k 10 120 python -u bench.py --png-only --no-cpu-baseline --images $n --distinct 1 > gpurun_out/sweep1/old$n.json 2> gpurun_out/sweep1/old$n.err
  python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print('old', sys.argv[2], r['roofline']['kernel_ms_per_launch'])" gpurun_out/sweep1/old$n.json $n
done

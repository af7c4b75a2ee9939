set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5t
for l in 1 4 16; do
JB_POOL_LPR=$l timeout -k 10 300 python tools/bench_engine_records.py --engines recommender_default > gpurun_out/r5t/eng_$l.json 2>gpurun_out/r5t/eng_$l.err || exit 1
echo "lpr $l"; python3 -c "import json; d=json.load(open('gpurun_out/r5t/eng_$l.json'))['recommender_default']; print(d['similar_row_from_datum_p50_us'], d['similar_row_from_datum_per_s'])"
done

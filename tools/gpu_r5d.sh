set -o pipefail
export TMPDIR=/tmp
R=/root/repo
mkdir -p $R/gpurun_out/r5d
timeout -k 10 200 python tools/prof_cluster.py --method gmm > gpurun_out/r5d/gmm.log 2>&1; echo "gmm rc=$?"
timeout -k 10 200 python tools/prof_cluster.py --method kmeans > gpurun_out/r5d/kmeans.log 2>&1; echo "kmeans rc=$?"
cat gpurun_out/r5d/gmm.log gpurun_out/r5d/kmeans.log
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktc -o run -- python3 $R/tools/prof_cluster.py --method gmm --points 50000 > $R/gpurun_out/r5d/ktc.log 2>&1; echo "ktc rc=$?"
find /tmp/ktc -name "*kernel_stats*" | head -5 > $R/gpurun_out/r5d/ktc_files.txt
i=0; for f in $(find /tmp/ktc -name "*kernel_stats*"); do i=$((i+1)); cp $f $R/gpurun_out/r5d/kstats_$i.csv; done
cd $R && tail -c 3000 gpurun_out/r5d/ktc.log > gpurun_out/r5d/ktc.tail && rm gpurun_out/r5d/ktc.log

# --inner hypre at the metric's N=59 (BoomerAMG on the s block; default np = 1 since round 5)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
mkdir -p gpurun_out/r5
timeout -k 10 500 python -u bench.py --inner hypre --steps 3 --warmup 1 --no-cpu --no-copy-probe --opt pls.amg_view=1 > gpurun_out/r5/hyp59.log 2>&1 || exit 1
grep "boomeramg\|setup\|warmup" gpurun_out/r5/hyp59.log | cut -c1-300; grep '^{' gpurun_out/r5/hyp59.log | cut -c90-140
dir=$REPO/gpurun_out/r5/prof_amg59; rm -rf $dir; mkdir -p $dir
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$dir" -o run -- python3 "$REPO/bench.py" --inner hypre --steps 1 --warmup 1 --no-cpu --no-copy-probe > "$dir/stdout.log" 2>&1) || exit 1
rm -f $dir/run_kernel_trace.csv
python3 -c "
import csv
rows=list(csv.DictReader(open('$dir/run_kernel_stats.csv')))
for r in rows[:14]: print(r['Name'][:70], r['Calls'], 'avg us', round(float(r['AverageNs'])/1e3,1), r['Percentage'])"

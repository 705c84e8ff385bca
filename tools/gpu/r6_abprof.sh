set -o pipefail
# rocprofv3 --kernel-trace --stats of the C5 line (tools/prof_lines.py c5) for the built library and ALT (an alternate libdrandgpu.so)
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abprof
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o run -- python3 $R/tools/prof_lines.py c5 --calls 2 > $O/new.log 2>&1 || exit 1
DRAND_GPU_LIB=${ALT:?set ALT to the alternate library} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/alt -o run -- python3 $R/tools/prof_lines.py c5 --calls 2 > $O/alt.log 2>&1 || exit 1
for v in new alt; do f=$(find $O/$v -name "*kernel_stats.csv" | head -1); cp $f $O/${v}_stats.csv; rm -rf $O/$v; done

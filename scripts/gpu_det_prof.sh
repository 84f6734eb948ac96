# rocprofv3 kernel trace of the detector with the round-3 defaults (persistent fused conv1..conv3,
# multi-row blob kernel): one detect pass in dispatch order plus per-kernel totals.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/detprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/scripts/video_layers.py 5 > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc = 0 ] || exit $rc
DB=$(find $O/prof -name "*.db" | head -1)
echo "db=$DB"
cd $R && python3 scripts/rocpd_kernels.py "$DB" --sequence blob_bilinear --end ssd_merge > $O/seq.txt 2>&1
echo "rocpd rc=$?"

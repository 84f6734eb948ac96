# Training CLI on RCCL with 2 peers sharing one GPU (one NCCL_HOSTID per rank): elastic local-SGD
# with top-k compression and checkpoints, then a resume from the last checkpoint; then the
# sharded trainer with PowerSGD. Each step under its own time limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/train_rccl
rm -rf $O /tmp/vcx_train_ck && mkdir -p $O
L="python -u scripts/rccl_rehearsal_launch.py --nproc 2 --timeout 200"
T="python -u -m distributedvolunteercomputing_amd.cli.main train --model gpt2-tiny --batch 4 --seq 128 --backend nccl --log-every 5"
timeout -k 10 230 $L --log-dir $O/a -- $T --elastic --steps 20 --compression topk --ckpt-dir /tmp/vcx_train_ck --ckpt-every 10 --store-port 29711 &&
echo "[train] phase a ok" &&
timeout -k 10 230 $L --log-dir $O/b -- $T --elastic --steps 30 --compression topk --ckpt-dir /tmp/vcx_train_ck --resume --store-port 29712 &&
echo "[train] phase b (resume) ok" &&
timeout -k 10 230 $L --log-dir $O/c -- $T --trainer sharded --replicas 1 --elastic --steps 12 --compression powersgd --store-port 29713 &&
echo "[train] phase c (sharded) ok"
rc=$?
ls /tmp/vcx_train_ck > $O/ckpt_ls.txt 2>&1
exit $rc

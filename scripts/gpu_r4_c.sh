# round 4, GPU call C: the 8-peer elastic rehearsals (one peer killed inside the all-to-all; kill 2 then rejoin)
cd $GRAFT_REPO_ROOT && ONLY="drop_collective_n8 drop_kill2_rejoin_n8" timeout -k 10 1000 bash scripts/gpu_rccl8_rehearsal.sh

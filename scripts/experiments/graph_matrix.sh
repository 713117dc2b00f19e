export HSA_ENABLE_IPC_MODE_LEGACY=0
for mode in 0 1 2; do for mix in 1 0; do
  VIP_SHARD_CAPTURE_MODE=$mode NCCL_GRAPH_MIXING_SUPPORT=$mix timeout -k 10 60 python scripts/experiments/graph_probe.py > gpurun_out/gp_${mode}_${mix}.txt 2>&1
  echo "mode=$mode mixing=$mix rc=$? $(grep -c 'equal = True' gpurun_out/gp_${mode}_${mix}.txt) rounds equal"
done; done

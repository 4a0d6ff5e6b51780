#!/bin/bash
# Round 5: which HIP call in bg_batch_execute blocks once torch's HIP runtime is loaded
# (BG_EXEC_TIMING), then the s_wakeup + put_op-guard variant run once.
set -o pipefail
out=gpurun_out/r05/${1:-exec}
mkdir -p $out
BG_EXEC_TIMING=1 timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 --rounds 12 > $out/p_plain.jsonl 2> $out/p_plain.err && \
BG_EXEC_TIMING=1 timeout -k 10 300 python -u tools/r05/h2h_probe.py --handles 4 --rounds 12 --torch > $out/p_torch.jsonl 2> $out/p_torch.err; exit $?
# the variant: the round-3 walker issuing s_wakeup after each posted miss, with the op-store guard
test -f biogarden_amd/variants/libbiogarden_gpu_wake1.so || { echo "variant .so missing" > $out/wake.txt; exit 2; }
cp biogarden_amd/libbiogarden_gpu.so /tmp/lib_tree.so || exit 3
cp biogarden_amd/variants/libbiogarden_gpu_wake1.so biogarden_amd/libbiogarden_gpu.so || exit 3
cmp -s biogarden_amd/libbiogarden_gpu.so biogarden_amd/variants/libbiogarden_gpu_wake1.so && echo "running the wake1 variant" > $out/wake.txt
timeout -k 10 200 python3 bench.py --no-cpu --no-h2h --no-affine --configs "" --R 8 --waves 16 --pipeline 1 \
  > $out/wake1.json 2> $out/wake1.err
rc=$?
echo "wake1 rc=$rc" >> $out/wake.txt
cp /tmp/lib_tree.so biogarden_amd/libbiogarden_gpu.so
exit 0

# BPLA items-kernel geometry sweep on C4: waves per workgroup, workgroups per
# CU, a variant library built with -DSK_BPLA_WPE=6 (third field, - = none)
# and the pairs a wave streams back to back (fourth field)
set -e
mkdir -p gpurun_out
for cfg in ${SWEEP:-16,1,-,1 16,1,-,2 16,1,-,3 16,1,-,4 16,1,-,6 12,2,6,2 12,2,6,3 8,2,-,3}; do
  IFS=, read w g v c <<< "$cfg"
  lib=""; [ "$v" != "-" ] && lib="$PWD/build_wpe$v/libstem_kernel_amd.so"
  tag=${w}_${g}_${v}_${c}
  SK_LIB_PATH=$lib SK_BPLA_IWAVES=$w SK_BPLA_IWG=$g SK_BPLA_CHUNK=$c timeout -k 10 120 python bench.py --config c4 --no-cpu-baseline --steps 20 --warmup 2 > gpurun_out/c4_$tag.log 2>&1
  echo "$cfg $(tail -1 gpurun_out/c4_$tag.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["roofline"]["kernel_ms_per_launch"])')" | tee -a gpurun_out/c4_sweep2.txt
done

set -o pipefail
R=$(pwd)
PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES;GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
  bash tools/pmc.sh r04e_c6 python3 $R/bench.py --config 6 --steps 2 --warmup 0 --primary-only --no-memo-off-run --no-pipelined-run --no-cpu-baseline --no-verify || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_r04e_c6 > gpurun_out/pmc_r04e_c6/summary.txt 2>&1 || true
grep -A12 "k_bpe_seg" gpurun_out/pmc_r04e_c6/summary.txt | head -30

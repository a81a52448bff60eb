# round 6: PMC of the 5x5 reprojection (288 -> 96 at 68 x 120, BM 96, halo) vs the g_s subpel conv shape
cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAIT_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum"
bash tools/gpu/pmc_probe.sh gpurun_out/pmc5a conv_x4_kernel "8 288 96 68 120 5 1 0" "$P1" "$P2" || exit 1
bash tools/gpu/pmc_probe.sh gpurun_out/pmc5b conv_x4_kernel "8 192 768 136 240 3 1 128" "$P1" "$P2"

set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05w; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-include-regex "k_sp_tile|k_sp_tupd" --kernel-trace --output-format csv -d $OUT/sq1 -o run -- python3 tools/tile_ab.py --one 100000 4 > $OUT/sq1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR --kernel-include-regex "k_sp_tile|k_sp_tupd" --kernel-trace --output-format csv -d $OUT/sq2 -o run -- python3 tools/tile_ab.py --one 100000 4 > $OUT/sq2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_sp_tile|k_sp_tupd" --kernel-trace --output-format csv -d $OUT/tcc -o run -- python3 tools/tile_ab.py --one 100000 4 > $OUT/tcc.log 2>&1

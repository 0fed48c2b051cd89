export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --kernel-trace -f csv -d gpurun_out/c4pmc -o run -- python scripts/legs.py config4one > gpurun_out/c4pmc.json 2> gpurun_out/c4pmc.log && echo pmc ok

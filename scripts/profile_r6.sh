#!/bin/bash
# Round-6 measurements behind profiles/r6/ (run on the GPU box from the repo root):
#   chainlat : dependent-issue latency of the quad chain's instructions
#              (tools/chainlat, one wave per SIMD)
#   qchain   : the quad compression chain itself, product form vs hand-
#              scheduled asm rounds (tools/qchain.hip), 1 and 4 waves per SIMD
#   c2_attrib: config 2's one-launch post split into ramp / prologue / DEK
#              wait / body / drain, beside the headline kernels' per-byte body
#              time (GLFSX_WGTIME build, scripts/c2_attrib.py)
#   c2_sq / c2_fetch / c2_write: PMC passes over config 2 (1 GiB at 2 MiB)
#   hl_sq    : the same SQ counters over the headline launches
#   concat   : Concat's per-slab host timeline (-DGLFSX_CONCAT_TRACE=1 build,
#              bash tools/build_variant.sh ctrace "-DGLFSX_CONCAT_TRACE=1") and its
#              kernel + memory-copy trace
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_r6}
mkdir -p $OUT
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
C2="python bench.py --no-extras --size-gib 1 --block-size 2097152 --steps 10 --warmup 2"
HL="python bench.py --no-extras --steps 3 --warmup 1"
timeout -k 10 60 ./tools/chainlat > $OUT/chainlat.json 2> $OUT/chainlat.err || exit $?
timeout -k 10 60 ./tools/qchain 256 256 > $OUT/qchain_1wave.json 2> $OUT/qchain.err || exit $?
timeout -k 10 60 ./tools/qchain 256 1024 > $OUT/qchain_4wave.json 2>> $OUT/qchain.err || exit $?
GLFSX_LIB=glfs_amd/libglfsx_wgtime.so timeout -k 10 200 python scripts/c2_attrib.py 3 > $OUT/c2_attrib.json 2> $OUT/c2_attrib.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace -f csv -d $OUT/c2_sq -o run -- $C2 > $OUT/c2_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/c2_fetch -o run -- $C2 > $OUT/c2_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/c2_write -o run -- $C2 > $OUT/c2_write.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc $SQ --kernel-trace -f csv -d $OUT/hl_sq -o run -- $HL > $OUT/hl_sq.log 2>&1 || exit $?
GLFSX_LIB=glfs_amd/libglfsx_ctrace.so timeout -k 10 200 python scripts/legs.py concat > $OUT/concat.json 2> $OUT/concat_trace.txt || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d $OUT/concat_tl -o run -- python scripts/legs.py concat > $OUT/concat_tl.json 2> $OUT/concat_tl.log || exit $?
python scripts/prof_summary.py $OUT $OUT/summary.json > $OUT/summary.txt
echo "profile ok"

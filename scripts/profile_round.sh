#!/bin/bash
# rocprofv3 evidence for one bench workload (run on the GPU box from the repo root):
#   kernel trace + stats of the bench command, then FETCH_SIZE, WRITE_SIZE and SQ counters in separate --pmc passes
# usage: bash scripts/profile_round.sh <tag> <bench args...>   -> gpurun_out/prof_<tag>/...
set -o pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o run -- python3 bench.py --no-cpu-baseline "$@" > $out/bench_under_trace.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 bench.py --no-cpu-baseline --no-end-to-end --steps 1 --warmup 0 "$@" > $out/fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 bench.py --no-cpu-baseline --no-end-to-end --steps 1 --warmup 0 "$@" > $out/write.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $out/sq -o run -- python3 bench.py --no-cpu-baseline --no-end-to-end --steps 1 --warmup 0 "$@" > $out/sq.log 2>&1 || exit $?
f=$(find $out/fetch -name '*counter_collection.csv' | head -1)
w=$(find $out/write -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_summary.py "$f" "$w" $out/pmc.json trace_pool_kernel,accumulate_kernel
python3 scripts/pmc_sq_summary.py "$(find $out/sq -name '*counter_collection.csv' | head -1)" $out/sq.json

#!/bin/bash
# Conditional-tape throughput including the chunk_map shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
exec tools/gpu_session.sh "cb:200:python -u tools/cond_bench.py > gpurun_out/cond_bench_s.jsonl"

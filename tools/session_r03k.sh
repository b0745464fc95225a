#!/bin/bash
# Staged encode with nontemporal scatter stores (key 27 = 3): parity of the
# staged kernels, config-4 A/B, and its WRITE counter.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
B="python3 $R/bench.py --config 4 --extra 0 --cpu-seconds 0 --no-host-inclusive --steps 4 --warmup 2"
PROF="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv --kernel-trace"
exec tools/gpu_session.sh \
  "t_nt:300:python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu $T -k 'staged_rm or staged_nt'" \
  "ab_nt:300:python -u tools/ab_knob.py --config 4 --key 27 --values 0,4 --rounds 5" \
  "wr_nt:200:export XDRG_TUNE=27=4 && $PROF --pmc WRITE_SIZE -d $R/gpurun_out/c4nt/write -o run -- $B"

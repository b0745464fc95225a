"""TEST INFRASTRUCTURE: a --test-codec whose rank 1 dies before its first
collective, so rank 0 blocks in the bench's barrier.  The launcher must end
the job with rank 1's status instead of waiting on rank 0 forever
(tests/test_bench_launcher.py)."""
import os
import sys


def make_workload(cfg, n, framed, rank):
    if rank == 1:
        sys.stderr.write("bench_fail_codec: rank 1 exits with status 3\n")
        sys.stderr.flush()
        os._exit(3)
    from bench_cpu_codec import make_workload as real
    return real(cfg, n, framed, rank)

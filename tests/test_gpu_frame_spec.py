"""The speculative record-mark walk (kernels_frame.hip k_fs_walk / k_fs_fix,
tuning key 47 = 1, the default) against the serial oracle
(oracle/xdr_oracle.c xo_frame_scan, RpcMessageParserTCP.isAllFragmentsArrived /
assembleXdr, rpc/RpcMessageParserTCP.java:63-140) and against the exact
kernels (key 47 = 0).

The walk guesses each 256 KiB super-chunk's entry and a chain per 64-word
segment; k_fs_fix checks every guess and walks wrong ones again, and gives
the stream to the exact kernels when it cannot settle it.  Its results must
be exact whatever the guesses do, so these streams aim at the guesses:
super-chunk boundaries inside marks and fragments, cut tails at and around
them, bodies of zeros, of small integers that read as plausible marks, and
of copies of real marks, fragments longer than a super-chunk, and a size
% 4 != 0 mark on the chain (the byte walk).  The shapes the bench runs
(framed configs 2 and 4) must settle without the exact kernels."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SUPER = 256 << 10   # bytes per super-chunk (kFSuper words)


@pytest.fixture(autouse=True)
def spec_default(gpu_ctx):
    gpu_ctx.tune(0)
    yield
    gpu_ctx.tune(0)


def _dev(b):
    if not b:
        return torch.zeros(4, dtype=torch.uint8, device="cuda")
    return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).cuda()


def scan(ctx, dev, n, cap):
    offs = torch.zeros(cap + 1, dtype=torch.int64, device="cuda")
    k = ctx.frame_scan(dev, n, offs, cap)
    return k, offs[:k + 1].cpu().tolist()


def check(ctx, stream, cap=1 << 22, deframe=True):
    """Spec walk == oracle (offsets, count), deframe bodies == oracle's; the
    exact kernels agree.  -> number of complete messages."""
    rc, want = oracle.frame_scan(stream, cap)
    dev = _dev(stream)
    k, got = scan(ctx, dev, len(stream), cap)
    assert k == len(want) - 1
    assert got == want
    if deframe:
        payload = torch.zeros(len(stream) + 16, dtype=torch.uint8, device="cuda")
        moffs = torch.zeros(cap + 1, dtype=torch.int64, device="cuda")
        k2, used = ctx.deframe(dev, len(stream), payload, payload.numel(), moffs, cap)
        assert k2 == k and used == want[-1]
    ctx.tune(47, 0)
    try:
        k3, got3 = scan(ctx, dev, len(stream), cap)
    finally:
        ctx.tune(0)
    assert (k3, got3) == (k, got)
    return k


def gave_up(ctx, fn):
    """-> (result of fn, speculative walks that gave up during it)."""
    g0 = ctx.internal_stat(2)
    r = fn()
    return r, ctx.internal_stat(2) - g0


def cfg2_stream(n, seed=1):
    words = np.random.default_rng(seed).integers(0, 2**32, (n, 9), dtype=np.uint64).astype(np.uint32)
    words[:, 0] = np.uint32(0x80000020).byteswap()
    return words.view(np.uint8).reshape(-1).tobytes()


def cfg4_stream(n, seed=2):
    """Record-marked configs[3] records: int32, string<8..256> (lowercase),
    int32<0..16> (bench.py's synthetic data), one fragment each."""
    rng = np.random.default_rng(seed)
    parts = []
    for _ in range(n):
        slen = int(rng.integers(8, 257))
        k = int(rng.integers(0, 17))
        s = rng.integers(97, 123, slen, dtype=np.uint8).tobytes() + b"\0" * (-slen % 4)
        body = (rng.integers(-2**31, 2**31 - 1, 1, dtype=np.int64).astype(">i4").tobytes()
                + np.array([slen], ">u4").tobytes() + s + np.array([k], ">u4").tobytes()
                + rng.integers(-2**31, 2**31 - 1, k, dtype=np.int64).astype(">i4").tobytes())
        parts.append(np.array([0x80000000 | len(body)], ">u4").tobytes() + body)
    return b"".join(parts)


def test_framed_cfg2_settles(gpu_ctx):
    n = 1 << 20
    s = cfg2_stream(n)
    (k, g) = gave_up(gpu_ctx, lambda: check(gpu_ctx, s, cap=n, deframe=False))
    assert k == n and g == 0


def test_framed_cfg4_settles(gpu_ctx):
    s = cfg4_stream(60000)
    (k, g) = gave_up(gpu_ctx, lambda: check(gpu_ctx, s))
    assert k == 60000 and g == 0


@pytest.mark.parametrize("which", ["cfg2", "cfg4"])
def test_cut_around_super_chunks(gpu_ctx, which):
    """Cut tails (STOP on the real chain) at and around super-chunk
    boundaries and inside the halo the entry guess walks."""
    s = cfg2_stream(40000, 3) if which == "cfg2" else cfg4_stream(16000, 4)
    cuts = []
    for b in range(SUPER, len(s), SUPER):
        cuts += [b - 513, b - 4, b - 1, b, b + 1, b + 3, b + 4, b + 37, b + 600]
    cuts += [4, 5, 36, 37, len(s) - 1, len(s) - 4]
    for cut in cuts:
        if 0 < cut <= len(s):
            check(gpu_ctx, s[:cut], deframe=False)


@pytest.mark.parametrize("body", ["zeros", "small-ints", "mark-copies", "last-flags"])
def test_bodies_that_read_as_marks(gpu_ctx, body):
    """Bodies whose words are plausible marks: the segment chains accepted
    first are false ones (exact results; the exact kernels may take over)."""
    rng = np.random.default_rng({"zeros": 1, "small-ints": 2, "mark-copies": 3, "last-flags": 4}[body])
    parts, nmsg = [], 0
    while sum(map(len, parts)) < 3 * SUPER + 12345:
        n = int(rng.integers(0, 200)) * 4
        if body == "zeros":
            b = bytes(n)
        elif body == "small-ints":
            b = (rng.integers(0, 64, n // 4, dtype=np.uint32) * 4).astype(">u4").tobytes()
        elif body == "mark-copies":   # words equal to this message's own mark
            b = np.full(n // 4, 0x80000000 | n, ">u4").tobytes()
        else:                          # LAST marks of small sizes
            b = (0x80000000 | rng.integers(0, 32, n // 4, dtype=np.uint32) * 4).astype(">u4").tobytes()
        parts.append(oracle.fragment(b, int(rng.choice([4, 64, 1 << 20]))))
        nmsg += 1
    s = b"".join(parts)
    assert check(gpu_ctx, s) == nmsg
    for cut in (SUPER, SUPER + 8, 2 * SUPER - 4):
        check(gpu_ctx, s[:cut], deframe=False)


def test_fragments_longer_than_a_super_chunk(gpu_ctx):
    """A 600 KiB fragment between small messages: super-chunks the chain
    jumps over (the entry checks fail; re-walked or the exact kernels)."""
    rng = np.random.default_rng(7)
    small = cfg2_stream(9000, 8)
    big = oracle.fragment(rng.integers(0, 256, 600 << 10, dtype=np.uint8).tobytes(), 1 << 30)
    s = small + big + small + big + big + small
    k = check(gpu_ctx, s)
    assert k == 3 * 9000 + 3


def test_one_skip_is_rewalked(gpu_ctx):
    """A 300 KiB fragment: the super-chunk it covers fails its entry check and
    is walked again (k_fs_fix), without the exact kernels."""
    rng = np.random.default_rng(17)
    small = cfg2_stream(20000, 18)
    big = oracle.fragment(rng.integers(0, 256, 300 << 10, dtype=np.uint8).tobytes(), 1 << 30)
    w0 = gpu_ctx.internal_stat(3)
    (k, g) = gave_up(gpu_ctx, lambda: check(gpu_ctx, small + big + small))
    assert k == 40001 and g == 0
    assert gpu_ctx.internal_stat(3) > w0


def test_unaligned_mark_on_the_chain(gpu_ctx):
    """A 6-byte fragment in the middle: the word walk meets a size % 4 != 0
    mark and the byte walk takes over, with the same results."""
    s = cfg2_stream(30000, 9)
    mid = oracle.fragment(b"abcdef", 6)
    k = check(gpu_ctx, s + mid + s)
    assert k == 60001


@pytest.mark.parametrize("seed", range(6))
def test_random_shapes_vs_exact(gpu_ctx, seed):
    """Re-fragmented messages of 0..2 KiB (fragments 4 B .. 4 KiB), several
    super-chunks, against the oracle and the exact kernels."""
    rng = np.random.default_rng(100 + seed)
    parts, nmsg = [], 0
    while sum(map(len, parts)) < 5 * SUPER:
        n = int(rng.integers(0, 512)) * 4
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        parts.append(oracle.fragment(b, int(rng.choice([4, 16, 256, 4096]))))
        nmsg += 1
    s = b"".join(parts)
    assert check(gpu_ctx, s) == nmsg

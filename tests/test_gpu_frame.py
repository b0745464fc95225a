"""Parallel record-mark walk (kernels_frame.hip):
xdrg_frame_scan and xdrg_deframe against the serial oracle (oracle/xdr_oracle.c
xo_frame_scan, a restatement of RpcMessageParserTCP.isAllFragmentsArrived /
assembleXdr, rpc/RpcMessageParserTCP.java:63-140) and the golden framing
fixtures.  Streams span several 1 MiB super-chunks, carry fragments of many
sizes (the re-fragmenter of ctest/rpc/RpcMessageParserTCPTest.java:161-181,
oracle.fragment), bodies full of small integers that look like marks, cut
tails, and fragment sizes that are not multiples of 4 (the byte-position
walk; the serial walk that a stream not 4-byte aligned takes must agree)."""
import numpy as np
import pytest

import gold
import oracle

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(autouse=True, params=[(1, 1), (4, 1), (7, 1), (4, 0)], ids=lambda v: f"emit{v[0]}-{'wave' if v[1] else 'pair'}")
def emit_per(request, gpu_ctx):
    """Sub-chunks per emit block (tuning key 36; 7 leaves a partial last
    block) and the emit kernel (key 48: a wave per sub-chunk, or k_fr_emit's
    two waves)."""
    gpu_ctx.tune(36, request.param[0])
    gpu_ctx.tune(48, request.param[1])
    yield request.param
    gpu_ctx.tune(0)


def _dev(b):
    if not b:
        return torch.zeros(4, dtype=torch.uint8, device="cuda")
    return torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).cuda()


def _dev_at(b, shift):
    """(address, owner): the stream `shift` bytes past a 16-byte boundary
    (a stream that is not 4-byte aligned takes the serial walk)."""
    t = torch.zeros(len(b) + 16, dtype=torch.uint8, device="cuda")
    if b:
        t[shift:shift + len(b)] = torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).cuda()
    return t.data_ptr() + shift, t


def build(rng, nmsg, aligned=True, big=0, marks_in_body=False):
    """-> (stream, bodies): nmsg messages, each re-fragmented."""
    bodies, parts = [], []
    for i in range(nmsg):
        n = int(rng.integers(0, 400))
        if aligned:
            n &= ~3
        if big and i % max(nmsg // big, 1) == 7:
            n = int(rng.integers(1 << 20, 3 << 20)) & ~3
        if marks_in_body:   # small BE ints everywhere: false chains through every body
            body = (rng.integers(0, 12, (n + 3) // 4, dtype=np.uint32) * 4).astype(">u4").tobytes()[:n]
        else:
            body = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        frag = int(rng.choice([4, 16, 64, 1024, 1 << 16, 1 << 22]))
        if not aligned:
            frag += int(rng.integers(0, 4))
        bodies.append(body)
        parts.append(oracle.fragment(body, frag))
    return b"".join(parts), bodies


def check(ctx, stream, bodies_all=None, cap=1 << 22, shift=0):
    rc, want = oracle.frame_scan(stream, cap)
    k_want = len(want) - 1
    dev, _owner = _dev_at(stream, shift) if shift else (_dev(stream), None)
    offs = torch.zeros(cap + 1, dtype=torch.int64, device="cuda")
    k = ctx.frame_scan(dev, len(stream), offs, cap)
    assert k == k_want
    assert offs[:k + 1].cpu().tolist() == want
    # assembled bodies
    payload = torch.zeros(len(stream) + 16, dtype=torch.uint8, device="cuda")
    moffs = torch.zeros(cap + 1, dtype=torch.int64, device="cuda")
    k2, used = ctx.deframe(dev, len(stream), payload, payload.numel(), moffs, cap)
    assert k2 == k_want and used == want[-1]
    mo = moffs[:k2 + 1].cpu().numpy()
    pl = payload[:int(mo[-1]) if k2 else 0].cpu().numpy().tobytes()
    got = [pl[mo[i]:mo[i + 1]] for i in range(k2)]
    if bodies_all is not None:
        assert got == bodies_all[:k2]
    return k, got


def test_golden_framing_deframe(gpu_ctx):
    for case in gold.load("framing.json")["cases"]:
        stream = bytes.fromhex(case["stream"])
        k, got = check(gpu_ctx, stream, cap=16)
        assert k == case["complete"]
        assert [g.hex() for g in got] == case["messages"]


@pytest.mark.parametrize("marks_in_body", [False, True], ids=["random-bodies", "mark-like-bodies"])
def test_parallel_walk_many_messages(gpu_ctx, marks_in_body):
    rng = np.random.default_rng(11 + marks_in_body)
    stream, bodies = build(rng, 30000, big=3, marks_in_body=marks_in_body)
    assert len(stream) > (8 << 20)   # several 1 MiB super-chunks
    k, _ = check(gpu_ctx, stream, bodies)
    assert k == len(bodies)


def test_parallel_walk_cut_tails(gpu_ctx):
    rng = np.random.default_rng(5)
    stream, bodies = build(rng, 6000, big=1)
    for cut in [3, 4, 5, len(stream) // 3, len(stream) // 2 + 1, len(stream) - 1, len(stream) - 4]:
        check(gpu_ctx, stream[:cut], bodies)


@pytest.mark.parametrize("shift", [0, 1, 3], ids=["byte_walk", "serial_walk1", "serial_walk3"])
def test_unaligned_fragment_sizes(gpu_ctx, shift):
    """Fragment sizes % 4 != 0: the parallel byte-position walk (an aligned
    stream) and the serial walk (a stream 1 or 3 bytes off alignment)."""
    rng = np.random.default_rng(8)
    stream, bodies = build(rng, 3000, aligned=False)
    k, _ = check(gpu_ctx, stream, bodies, shift=shift)
    assert k == len(bodies)


@pytest.mark.parametrize("shift", [0, 1], ids=["byte_walk", "serial_walk"])
@pytest.mark.parametrize("marks_in_body", [False, True], ids=["random-bodies", "mark-like-bodies"])
def test_byte_walk_many_messages(gpu_ctx, shift, marks_in_body):
    """Several byte-mode super-chunks (64 KiB each), big fragments, bodies of
    small integers (false chains at every byte offset)."""
    rng = np.random.default_rng(21 + marks_in_body)
    stream, bodies = build(rng, 8000, aligned=False, big=2, marks_in_body=marks_in_body)
    k, _ = check(gpu_ctx, stream, bodies, shift=shift)
    assert k == len(bodies)


@pytest.mark.parametrize("shift", [0, 2], ids=["byte_walk", "serial_walk"])
def test_byte_walk_cut_tails(gpu_ctx, shift):
    rng = np.random.default_rng(6)
    stream, bodies = build(rng, 2000, aligned=False)
    for cut in [5, 6, 7, len(stream) // 3, len(stream) // 2 + 1, len(stream) - 1, len(stream) - 2, len(stream) - 5]:
        check(gpu_ctx, stream[:cut], bodies, shift=shift)


@pytest.mark.parametrize("shift", [0, 3], ids=["byte_walk", "serial_walk"])
def test_one_odd_fragment_then_aligned(gpu_ctx, shift):
    """The bench's serial-cliff shape: a 3-byte fragment, then aligned
    messages (every later mark at byte offset 3 mod 4)."""
    rng = np.random.default_rng(9)
    stream, bodies = build(rng, 4000)
    head = oracle.fragment(b"abc", 3)
    k, _ = check(gpu_ctx, head + stream, [b"abc"] + bodies, shift=shift)
    assert k == len(bodies) + 1


@pytest.mark.parametrize("shift", [0, 1], ids=["byte_walk", "serial_walk"])
def test_byte_walk_cap(gpu_ctx, shift):
    rng = np.random.default_rng(12)
    stream, bodies = build(rng, 700, aligned=False)
    for cap in (1, 7, 300):
        check(gpu_ctx, stream, bodies, cap=cap, shift=shift)


def test_cap_limits_messages(gpu_ctx):
    rng = np.random.default_rng(2)
    stream, bodies = build(rng, 500)
    rc, want = oracle.frame_scan(stream, 10)
    dev = _dev(stream)
    payload = torch.zeros(len(stream), dtype=torch.uint8, device="cuda")
    moffs = torch.zeros(11, dtype=torch.int64, device="cuda")
    k, used = gpu_ctx.deframe(dev, len(stream), payload, payload.numel(), moffs, 10)
    assert k == 10 and used == want[-1]
    mo = moffs.cpu().numpy()
    pl = payload[:int(mo[-1])].cpu().numpy().tobytes()
    assert [pl[mo[i]:mo[i + 1]] for i in range(10)] == bodies[:10]


def test_payload_capacity(gpu_ctx):
    from oncrpc4j_amd import engine
    stream, bodies = build(np.random.default_rng(4), 50)
    need = sum(len(b) for b in bodies)
    payload = torch.zeros(need, dtype=torch.uint8, device="cuda")
    moffs = torch.zeros(51, dtype=torch.int64, device="cuda")
    with pytest.raises(engine.CapacityError):
        gpu_ctx.deframe(_dev(stream), len(stream), payload, need - 1, moffs, 50)
    assert not payload.any()


def test_framed_cfg2_stream_offsets(gpu_ctx):
    """A record-marked configs[1] stream (36-byte messages): offsets 36 i."""
    n = 1 << 20
    words = np.random.default_rng(1).integers(0, 2**32, (n, 9), dtype=np.uint64).astype(np.uint32)
    words[:, 0] = np.uint32(0x80000020).byteswap()
    dev = torch.from_numpy(words.view(np.uint8).reshape(-1)).cuda()
    offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    k = gpu_ctx.frame_scan(dev, 36 * n, offs, n)
    assert k == n
    assert torch.equal(offs, torch.arange(0, 36 * (n + 1), 36, dtype=torch.int64, device="cuda"))

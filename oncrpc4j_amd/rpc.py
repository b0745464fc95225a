"""rpc.py — batches of ONC RPC messages on the XDR engine.

The XDR hot path's real callers are the RPC message layer.  Paths below are
relative to /root/reference/oncrpc4j-core/src/main/java/org/dcache/oncrpc4j/.

* Server send side, RpcCall.acceptedReply (rpc/RpcCall.java:323-343): every
  reply is xid, REPLY, MSG_ACCEPTED, the verifier (flavour + opaque<> body,
  rpc/RpcAuthVerifier.java:58-61), accept_stat, then the XdrAble body, sent
  as one record-marked TCP message (grizzly/GrizzlyRpcTransport.java:97-124).
  ReplyEncoder turns N such replies of one body schema into ONE device batch:
  the prelude words that are the same in every reply are constant columns
  (XDRG_STRIDE_CONST), the xids a column, the bodies the caller's columns.
* Server receive side, RpcProtocolFilter.handleRead (rpc/RpcProtocolFilter.java:
  51-54) + RpcCall.accept (rpc/RpcCall.java:206-216) + RpcCredential.decode
  (rpc/RpcCredential.java:29-55): xid, msg_type, rpcvers, prog, vers, proc,
  credential, verifier, then the procedure's arguments.  CallDecoder decodes
  the headers of a batch of calls (to group them by procedure), then a group
  of calls of one procedure with its argument schema, and checks msg_type /
  rpcvers / credential flavour on the device as the reference does per call.
* Client receive side, RpcReply (rpc/RpcReply.java:48-63): reply_stat,
  verifier, accept_stat, then the result — ReplyDecoder for accepted replies.

The field tapes follow the reference's call order exactly, so the bytes are
the reference's; everything compute-side runs in libxdrgpu.so.  torch is the
device allocator and does the vectorised header checks.
"""
from . import abi, engine

# rpc/RpcMessageType.java:27-28, rpc/RpcReplyStatus.java:32-37,
# rpc/RpcAccepsStatus.java:33-53, rpc/RpcAuthType.java:31-46, rpc/RpcCall.java:62
CALL, REPLY = 0, 1
MSG_ACCEPTED, MSG_DENIED = 0, 1
SUCCESS, PROG_UNAVAIL, PROG_MISMATCH, PROC_UNAVAIL, GARBAGE_ARGS, SYSTEM_ERR = 0, 1, 2, 3, 4, 5
AUTH_NONE, AUTH_UNIX, RPCSEC_GSS, AUTH_TLS = 0, 1, 6, 7
RPCVERS = 2

INT = (abi.T_INT, abi.K_SCALAR, 0)
OPAQUE_DYN = (abi.T_OPAQUE, abi.K_DYNAMIC, 0)
STRING_DYN = (abi.T_STRING, abi.K_DYNAMIC, 0)
INT_DYN = (abi.T_INT, abi.K_DYNAMIC, 0)

# ---- field tapes ---------------------------------------------------------------
# accepted reply prelude: xid, msg_type, reply_stat, verifier flavour, verifier
# body, accept_stat (RpcCall.java:328-332).  With AUTH_NONE's empty verifier
# body the opaque<> is its zero length word, the same 4 bytes as an int 0.
REPLY_PRELUDE_NONE = [INT, INT, INT, INT, INT, INT]
REPLY_PRELUDE = [INT, INT, INT, INT, OPAQUE_DYN, INT]

# call header up to the credential (RpcCall.java:462-467 on the client side)
CALL_HEADER = [INT] * 6               # xid, msg_type, rpcvers, prog, vers, proc
CRED_NONE = [INT, OPAQUE_DYN]         # flavour, body (RpcAuthTypeNone.java:69-77)
# AUTH_UNIX (RpcAuthTypeUnix.java:71-79, 123-131): flavour, body length, stamp,
# machine name, uid, gid, gids<>
CRED_UNIX = [INT, INT, INT, STRING_DYN, INT, INT, INT_DYN]
VERIFIER = [INT, OPAQUE_DYN]          # RpcAuthVerifier.java:53-61

CREDENTIALS = {AUTH_NONE: CRED_NONE, AUTH_UNIX: CRED_UNIX}

# field index of each header item in a decoded call
XID, MSG_TYPE, RPC_VERS, PROG, VERS, PROC, CRED_FLAVOR = range(7)


def accepted_reply_fields(body_fields, verifier_body=False):
    """Field tape of one accepted reply (RpcCall.java:328-333)."""
    return (REPLY_PRELUDE if verifier_body else REPLY_PRELUDE_NONE) + [tuple(f) for f in body_fields]


def call_fields(flavor, args_fields=()):
    """Field tape of one call with credential `flavor` (AUTH_NONE / AUTH_UNIX)
    and an AUTH_NONE-shaped verifier, then the arguments."""
    if flavor not in CREDENTIALS:
        raise ValueError(f"credential flavour {flavor} has no batch tape")
    return CALL_HEADER + CREDENTIALS[flavor] + VERIFIER + [tuple(f) for f in args_fields]


def _dev(ctx):
    return f"cuda:{ctx.device}"


class ReplyEncoder:
    """N calls' RpcCall.reply(body) / acceptedReply(stat, body) as one batch.

    Every reply carries xid[i]; accept_stat is a constant (SUCCESS by default)
    or a per-reply int32 tensor; the verifier is AUTH_NONE (constant) unless
    verifier_body=True, when each reply takes (values, offsets) opaque<>
    bodies with the constant flavour `verifier_flavor`.  framed=True prepends
    the TCP record mark of GrizzlyRpcTransport.java:103-110 (UDP: False)."""

    def __init__(self, ctx, body_fields, accept_stat=SUCCESS, verifier_flavor=AUTH_NONE,
                 verifier_body=False, framed=True):
        import torch
        self.ctx = ctx
        self.framed = framed
        self.verifier_body = verifier_body
        self.body_fields = [tuple(f) for f in body_fields]
        self.fields = accepted_reply_fields(self.body_fields, verifier_body)
        self.schema = engine.Schema(self.fields)
        # constant words: msg_type, reply_stat, verifier flavour, empty verifier length, accept_stat
        self._const = torch.tensor([REPLY, MSG_ACCEPTED, verifier_flavor, 0, accept_stat],
                                   dtype=torch.int32, device=_dev(ctx))

    def _col(self, i):
        return (self._const.data_ptr() + 4 * i, abi.STRIDE_CONST, None, 0)

    def columns(self, xids, body_cols, verifier=None, accept_stats=None):
        cols = [(xids, 4, None, 0), self._col(0), self._col(1), self._col(2)]
        if self.verifier_body:
            if verifier is None:
                raise ValueError("verifier_body=True needs (values, offsets) verifier bodies")
            vals, offs = verifier
            cols.append((vals, 0, offs, vals.numel()))
        else:
            cols.append(self._col(3))
        cols.append((accept_stats, 4, None, 0) if accept_stats is not None else self._col(4))
        if len(body_cols) != len(self.body_fields):
            raise ValueError("one column per body field")
        return cols + list(body_cols)

    def encode(self, xids, body_cols, n, out, out_cap, rec_offsets=None, verifier=None,
               accept_stats=None, async_=False, out_len=None):
        """-> bytes written (sync mode).  xids: int32 device tensor [n]."""
        if xids.numel() < n:
            raise ValueError("need one xid per reply")
        return self.ctx.encode(self.schema, self.columns(xids, body_cols, verifier, accept_stats), n,
                               out, out_cap, rec_offsets=rec_offsets, framed=self.framed,
                               async_=async_, out_len=out_len)


class CallDecoder:
    """Batches of incoming calls (RpcProtocolFilter.handleRead + RpcCall.accept).

    decode_headers() reads xid .. proc of every message (the rest of each
    extent stays unread), so the caller can group calls by (prog, vers,
    proc); decode() reads whole calls of one credential flavour and one
    argument schema.  check() flags what the reference would not dispatch:
    a non-CALL message (RpcProtocolFilter.java:63-84), rpcvers != 2
    (RpcMismatchReply, RpcCall.java:208-210) and a credential flavour other
    than the batch's (RpcCredential.java:33-52 picks the decoder per call)."""

    def __init__(self, ctx, framed=True):
        self.ctx = ctx
        self.framed = framed
        self._hdr_schema = engine.Schema(CALL_HEADER + [INT])

    def decode_headers(self, xdr, xdr_len, n, rec_offsets):
        """-> int32 device tensor [n, 7] (xid, msg_type, rpcvers, prog, vers,
        proc, credential flavour) and (status, first_bad, err)."""
        import torch
        hdr = torch.zeros((n, 7), dtype=torch.int32, device=_dev(self.ctx))
        cols = [(hdr.data_ptr() + 4 * k, 28, None, 0) for k in range(7)]
        st = self.ctx.decode(self._hdr_schema, xdr, xdr_len, n, cols, rec_offsets=rec_offsets,
                             framed=self.framed, raise_on_error=False)
        return hdr, st

    def decode(self, flavor, args_fields, xdr, xdr_len, n, rec_offsets, dyn_caps):
        """Decode n whole calls -> (DeviceBatch of call_fields(flavor, args_fields),
        (status, first_bad, err)).  dyn_caps[k]: element capacity of dynamic field k."""
        from .columns import DeviceBatch
        fields = call_fields(flavor, args_fields)
        batch = DeviceBatch.empty(fields, n, dyn_caps, device=_dev(self.ctx))
        st = self.ctx.decode(engine.Schema(fields), xdr, xdr_len, n, batch.columns(),
                             rec_offsets=rec_offsets, framed=self.framed, raise_on_error=False)
        return batch, st

    @staticmethod
    def check(headers):
        """Vectorised RpcProtocolFilter / RpcCall.accept checks -> bool device masks [n]:
        not_call (a REPLY or junk type), rpc_mismatch (rpcvers != 2),
        unsupported_flavor (no batch tape for the credential)."""
        import torch
        fl = headers[:, CRED_FLAVOR]
        known = torch.zeros_like(fl, dtype=torch.bool)
        for f in CREDENTIALS:
            known |= fl == f
        return {"not_call": headers[:, MSG_TYPE] != CALL,
                "rpc_mismatch": headers[:, RPC_VERS] != RPCVERS,
                "unsupported_flavor": ~known}

    @staticmethod
    def group_by_procedure(headers):
        """(prog, vers, proc, credential flavour) -> int64 record indices, one
        batch per group (each group decodes with one field tape)."""
        import torch
        key = headers[:, PROG:CRED_FLAVOR + 1].to(torch.int64)
        uniq, inv = torch.unique(key, dim=0, return_inverse=True)
        order = torch.argsort(inv, stable=True)
        counts = torch.bincount(inv, minlength=uniq.shape[0]).tolist()
        groups, pos = {}, 0
        for u, c in zip(uniq.tolist(), counts):
            groups[tuple(u)] = order[pos:pos + c]
            pos += c
        return groups


class ReplyDecoder:
    """Client side: accepted replies of one result schema (RpcReply.java:48-63
    + the result's xdrDecode, RpcReply.java:112)."""

    def __init__(self, ctx, body_fields, framed=True):
        self.ctx = ctx
        self.framed = framed
        self.fields = accepted_reply_fields(body_fields, verifier_body=True)
        self.schema = engine.Schema(self.fields)

    def decode(self, xdr, xdr_len, n, rec_offsets, dyn_caps):
        from .columns import DeviceBatch
        batch = DeviceBatch.empty(self.fields, n, dyn_caps, device=_dev(self.ctx))
        st = self.ctx.decode(self.schema, xdr, xdr_len, n, batch.columns(), rec_offsets=rec_offsets,
                             framed=self.framed, raise_on_error=False)
        return batch, st

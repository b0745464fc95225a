"""oncrpc4j_amd — MI355X-native XDR encode/decode engine for the oncrpc4j hot path.

The hot path of dCache/oncrpc4j that this package replaces is
org.dcache.oncrpc4j.xdr.Xdr (XDR encode/decode, RFC 4506) plus RFC 1831
record-mark framing (GrizzlyRpcTransport / RpcMessageParserTCP).  The compute
lives in libxdrgpu.so (hand-written HIP for gfx950, C-ABI in include/xdrg.h);
this package is the Python host side above that ABI.
"""
from . import abi  # noqa: F401

__all__ = ["abi", "engine", "columns", "parallel", "rpc", "rpcgen"]

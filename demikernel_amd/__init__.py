"""demikernel_amd — MI355X-native receive path for Demikernel's inetstack.

One hot path, rebuilt for gfx950: per-frame Ethernet/IPv4/TCP/UDP parse, the one's-complement Internet checksums and
the 4-tuple socket demux, run as hand-written HIP kernels over HBM-resident frame batches behind a C ABI
(include/dk_rx.h, libdk_rx.so). See DESIGN.md and INTEGRATION.md.
"""
from .rx import (  # noqa: F401
    Comm,
    Config,
    Fail,
    FrameBatch,
    RxEngine,
    RxResults,
    SocketId,
    V,
    VERDICTS,
    flow_array,
    ipv4,
    ipv4_str,
    raise_for_verdict,
    tx_tuning,
)

__all__ = ["Comm", "Config", "Fail", "FrameBatch", "RxEngine", "RxResults", "SocketId", "V", "VERDICTS", "flow_array",
           "ipv4", "ipv4_str", "raise_for_verdict", "tx_tuning"]

"""The drop-in boundary on CPU: libdk_rx.so loads, exports every function include/*.h declares, the ctypes mirror
matches the C layout, and the verdict/errno tables match the reference's errno per check. No compute calls."""
import ctypes
import os
import re
import subprocess

import pytest

from demikernel_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("dk_rx.h", "dk_diag.h", "dk_ring.h", "dk_tcp.h", "dk_demi.h", "dk_comm.h")]


def declared_functions(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.findall(r"^[a-z_][\w \*]*?\b(dk_\w+)\s*\(", src, flags=re.M)


def test_headers_compile_as_c_and_cxx(tmp_path):
    for h in HEADERS:
        for lang, std in (("c", "-std=c99"), ("c++", "-std=c++11")):
            subprocess.run(["gcc", "-x", lang, std, "-Wall", "-Werror", "-fsyntax-only", h], check=True)


def test_every_declared_function_is_exported():
    lib = N.load_library()
    names = set()
    for h in HEADERS:
        names |= set(declared_functions(h))
    assert {"dk_rx_process", "dk_rx_ctx_create", "dk_tx_checksum", "dk_diag_read_probe", "dk_rx_process_tpacket3",
            "dk_tcp_rx_process", "dk_rx_into_sgarrays", "dk_tcp_into_sgarrays", "dk_rx_flow_counts_allreduce",
            "dk_rx_flow_counts_allreduce_to",
            "dk_comm_init_rank"} <= names
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert names <= exported, names - exported
    bound = {f[0] for f in N.ALL_FUNCTIONS}
    assert bound == names, (names ^ bound)
    for n in names:
        getattr(lib, n)


def test_struct_layout_matches_ctypes(tmp_path):
    """sizeof/offsetof from the C compiler == the ctypes mirror (dk_rx_cfg, dk_flow, dk_rx_batch, dk_rx_results)."""
    structs = {"dk_rx_cfg": N.DkRxCfg, "dk_flow": N.DkFlow, "dk_rx_batch": N.DkRxBatch, "dk_rx_results": N.DkRxResults,
               "dk_tcp_view": N.DkTcpView, "dk_tcp_conn": N.DkTcpConn, "dk_tcp_out": N.DkTcpOut,
               "dk_demi_sgaseg_t": N.DemiSgaseg, "dk_demi_sgarray_t": N.DemiSgarray, "dk_tcp_opt": N.DkTcpOpt,
               "dk_tcp_opts": N.DkTcpOpts}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADERS[0]}"', f'#include "{HEADERS[3]}"',
             f'#include "{HEADERS[4]}"',
             "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-o", str(exe), str(c)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True, check=True)
               .stdout.splitlines())
    for cname, cls in structs.items():
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(cls, fname).offset, (cname, fname)
    assert ctypes.sizeof(N.DkFlow) == N.FLOW_DTYPE.itemsize == 16
    assert ctypes.sizeof(N.DkTcpConn) == N.CONN_DTYPE.itemsize == 288
    assert ctypes.sizeof(N.DkTcpOpts) == N.TCP_OPTS_DTYPE.itemsize == 96
    for fname, _ in N.DkTcpOpts._fields_:
        assert N.TCP_OPTS_DTYPE.fields[fname][1] == getattr(N.DkTcpOpts, fname).offset, fname
    for fname, _ in N.DkTcpConn._fields_:
        assert N.CONN_DTYPE.fields[fname][1] == getattr(N.DkTcpConn, fname).offset, fname


def test_tcp_header_constants():
    hdr = open(HEADERS[3]).read()
    for i, name in enumerate(N.TCP_ACTIONS):
        assert re.search(rf"DK_TCP_{name} = {i}[,\s]", hdr), name
    assert f"DK_TCP_OOO_MAX {N.DK_TCP_OOO_MAX}u" in hdr and f"DK_TCP_DELIV_EXTRA {N.DK_TCP_DELIV_EXTRA}u" in hdr
    for name, v in (("NONE", N.DK_TCP_NONE), ("ESTABLISHED", N.DK_TCP_ESTABLISHED), ("CLOSED", N.DK_TCP_CLOSED)):
        assert re.search(rf"DK_TCP_{name} = {v}", hdr), name


def test_defer_scope_constant():
    """The flow-table size up to which DK_RX_BATCH_DEFER_COUNTS defers flow counts: header == Python mirror (rx.py
    RxEngine.flow_counts_deferred, shard.py)."""
    hdr = open(HEADERS[0]).read()
    assert f"#define DK_RX_MAX_DEFERRED_FLOWS {N.DK_RX_MAX_DEFERRED_FLOWS}u" in hdr


def test_verdict_tables():
    lib = N.load_library()
    assert lib.dk_rx_abi_version() == 4
    bid = lib.dk_rx_build_id().decode()
    import __graft_entry__
    assert bid == __graft_entry__.tree_build_id(), (bid, "the loaded library is not this tree's build")
    for i, name in enumerate(N.VERDICTS):
        assert lib.dk_rx_verdict_name(i).decode() == name
    assert lib.dk_rx_verdict_name(N.DK_V_COUNT).decode() == "UNKNOWN"
    EBADMSG, ENOTSUP, EIO, EINVAL = 74, 95, 5, 22
    expect = {name: 0 for name in N.VERDICTS}
    for name in ("ETH_SHORT", "IP_SHORT", "IP_IHL_SMALL", "IP_HDR_TRUNC", "IP_TOTLEN_SMALL", "IP_TOTLEN_BIG",
                 "IP_EVIL", "IP_TTL", "IP_CSUM_FFFF", "IP_CSUM", "TCP_SHORT", "TCP_DOFF_TRUNC", "TCP_DOFF_SMALL",
                 "TCP_CSUM", "TCP_OPT", "UDP_SHORT", "UDP_LEN", "UDP_CSUM", "ARP_SHORT", "ICMP_SHORT", "ICMP_CSUM",
                 "ICMP_TYPE"):
        expect[name] = EBADMSG
    for name in ("ETH_TYPE", "IP_VERSION", "IP_MF", "IP_FRAGOFF", "IP_PROTO", "ARP_UNSUP"):
        expect[name] = ENOTSUP
    expect["TCP_OPT_EIO"] = EIO
    expect["BAD_DESC"] = EINVAL
    for i, name in enumerate(N.VERDICTS):
        assert lib.dk_rx_verdict_errno(i) == expect[name], name
    hdr = open(HEADERS[0]).read()
    for i, name in enumerate(N.VERDICTS):
        assert re.search(rf"DK_V_{name} = {i},", hdr), name
    assert f"DK_V_COUNT = {N.DK_V_COUNT}" in hdr


def test_single_hip_runtime_in_process():
    """torch's libamdhip64 and ours must be one runtime (see _native.load_library)."""
    N.load_library()
    import torch  # noqa: F401

    maps = open("/proc/self/maps").read()
    paths = {l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}
    assert len(paths) == 1, paths


def test_ctx_create_rejects_bad_device_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    lib = N.load_library()
    cfg = N.DkRxCfg(0, 0, 0, 0, 0)
    h = ctypes.c_void_p()
    assert lib.dk_rx_ctx_create(ctypes.byref(cfg), ctypes.byref(h)) == 22
    assert lib.dk_rx_ctx_create(None, ctypes.byref(h)) == 22


def test_demi_sgarray_layout_is_the_reference_abi():
    """dk_demi_sgarray_t has demi_sgarray_t's size and field offsets (include/demi/types.h:38-68, packed; the sizes
    tests/c/sizes.c:48-68 asserts: 12-byte segment, 40-byte array)."""
    assert ctypes.sizeof(N.DemiSgaseg) == 12 and ctypes.sizeof(N.DemiSgarray) == 40
    assert N.DemiSgarray.sga_numsegs.offset == 8 and N.DemiSgarray.sga_segs.offset == 12
    assert N.DemiSgarray.sga_addr.offset == 24


def test_into_sgarrays_matches_pop_semantics():
    """dk_rx_into_sgarrays over the oracle's results of a mixed batch: one array per delivered UDP datagram in frame
    order, one segment over the payload window, sga_buf = token, sga_addr = (AF_INET, sport, src_ip) in network order
    (libos.rs:495-499, pal/mod.rs:154-160); delivered TCP frames are not pops (dk_tcp_into_sgarrays); ENOSPC past cap.
    Host-only call."""
    import numpy as np

    from demikernel_amd import ipv4, synth
    from oracle.oracle import OraclePeer

    lib = N.load_library()
    flows = np.concatenate([synth.make_flows(32), synth.make_flows(16, kind="udp")])
    n = 600
    tr = synth.traffic(n, synth.imix_ip_lengths(n), flows, seed=3)
    blob, off, lens = synth.build_numpy(tr)
    synth.corrupt_numpy(blob, off, synth.corruption_plan(n, 0.2, tr))
    peer = OraclePeer(ipv4(synth.BOB_IPV4))
    peer.set_flows(flows)
    r = peer.process(blob, off, lens)
    meta, src, ports, pay = (np.ascontiguousarray(r[k], dtype=np.uint32) for k in ("meta", "src_ip", "ports", "payload"))
    tokens = (ctypes.c_void_p * n)(*[0x1000 + 16 * i for i in range(n)])
    out = (N.DemiSgarray * n)()
    idx = np.zeros(n, np.uint32)
    nout = ctypes.c_uint32()
    base = blob.ctypes.data
    off32 = off.astype(np.uint32)
    rc = lib.dk_rx_into_sgarrays(base, off32.ctypes.data, n, meta.ctypes.data, src.ctypes.data, ports.ctypes.data,
                                 pay.ctypes.data, tokens, out, idx.ctypes.data, n, ctypes.byref(nout))
    assert rc == 0
    v = meta & 0xFF
    deliv = np.nonzero(v == 1)[0]
    assert nout.value == len(deliv) > 0 and (v == 0).any()
    assert (idx[: nout.value] == deliv).all()
    for k, i in enumerate(deliv):
        s = out[k]
        assert s.sga_buf == 0x1000 + 16 * i and s.sga_numsegs == 1
        assert s.sga_segs[0].sgaseg_buf == base + int(off32[i]) + int(pay[i] & 0xFFFF)
        assert s.sga_segs[0].sgaseg_len == pay[i] >> 16
        assert s.sga_addr.sin_family == 2  # AF_INET
        assert s.sga_addr.sin_port == int.from_bytes(int(ports[i] & 0xFFFF).to_bytes(2, "big"), "little")
        assert s.sga_addr.sin_addr == src[i]
    # the delivered payload is what the frame carries after the strip (bytes S + hlen .. E)
    i = deliv[0]
    o, p = int(off32[i]), int(pay[i])
    assert ctypes.string_at(out[0].sga_segs[0].sgaseg_buf, p >> 16) == blob[o + (p & 0xFFFF): o + (p & 0xFFFF) + (p >> 16)].tobytes()
    # capacity: the first cap arrays, ENOSPC (errno 28)
    rc = lib.dk_rx_into_sgarrays(base, off32.ctypes.data, n, meta.ctypes.data, src.ctypes.data, ports.ctypes.data,
                                 pay.ctypes.data, None, out, None, 3, ctypes.byref(nout))
    assert rc == 28 and nout.value == 3 and out[0].sga_buf == base + int(off32[deliv[0]])
    assert lib.dk_rx_into_sgarrays(None, None, 0, None, None, None, None, None, None, None, 0, ctypes.byref(nout)) == 0
    assert lib.dk_rx_into_sgarrays(None, off32.ctypes.data, n, meta.ctypes.data, src.ctypes.data, ports.ctypes.data,
                                   pay.ctypes.data, None, out, None, n, ctypes.byref(nout)) == 22


def test_tcp_into_sgarrays_are_the_receive_queue():
    """dk_tcp_into_sgarrays over the oracle's dk_tcp results of a reordered stream with duplicates, strays and FINs
    (the GPU's are bit-exact to these, tests/test_gpu_tcp.py): per connection, one array per pushed buffer in queue
    order over exactly that buffer's bytes, zero address; FIN's EOF buffer is an empty segment; retransmitted and
    out-of-window bytes never appear (the delivered bytes add up to RCV.NXT's advance). Host-only call."""
    import numpy as np

    from demikernel_amd import ipv4, synth
    from oracle import oracle as O
    from oracle.oracle import OraclePeer

    lib = N.load_library()
    flows, tr, table = synth.tcp_streams(4000, 5, buffer_size=1 << 22, seed=77)
    blob, off, lens = synth.build_numpy(tr)
    peer = OraclePeer(ipv4(synth.BOB_IPV4))
    peer.set_flows(flows)
    rx = peer.process(blob, off, lens)
    t0 = table.copy()
    out = O.tcp_process(table, rx)
    n = len(off)
    off32 = np.ascontiguousarray(off, np.uint32)
    base = blob.ctypes.data
    arrs = (N.DemiSgarray * (n + 64))()
    nout = ctypes.c_uint32()
    dupes = 0
    for c in range(len(table)):
        if t0["state"][c] != N.DK_TCP_ESTABLISHED:
            continue
        a, k = int(out["deliv_start"][c]), int(out["deliv_count"][c])
        dv = np.ascontiguousarray(out["deliv"][a:a + k])
        rc = lib.dk_tcp_into_sgarrays(base, off32.ctypes.data, n, dv.ctypes.data, k, None, arrs, n + 64,
                                      ctypes.byref(nout))
        assert rc == 0 and nout.value == k
        total = 0
        for j in range(k):
            s, v = arrs[j], dv[j]
            assert s.sga_numsegs == 1 and bytes(s.sga_addr) == bytes(16)
            if v["ref"] == N.DK_TCP_REF_EOF:
                assert s.sga_buf is None and s.sga_segs[0].sgaseg_len == 0
                continue
            assert s.sga_buf == base + int(off32[v["ref"]])
            assert s.sga_segs[0].sgaseg_buf == base + int(off32[v["ref"]]) + int(v["off"])
            assert s.sga_segs[0].sgaseg_len == v["len"]
            total += int(v["len"])
        fin = int(np.any(dv["ref"] == N.DK_TCP_REF_EOF))
        assert (int(table["receive_next"][c]) - int(t0["receive_next"][c])) % 2**32 == total + fin, c
        dupes += int(((out["action"] == N.A["DUPLICATE"]) & (rx["flow_id"] == c)).sum())
    assert dupes > 0  # the stream had retransmissions, and none of their bytes were handed out
    # errors: a ref outside the batch, capacity
    dv = np.zeros(2, N.VIEW_DTYPE)
    dv["ref"] = [0, n]
    assert lib.dk_tcp_into_sgarrays(base, off32.ctypes.data, n, dv.ctypes.data, 2, None, arrs, 4, ctypes.byref(nout)) == 22
    dv["ref"] = [0, 1]
    assert lib.dk_tcp_into_sgarrays(base, off32.ctypes.data, n, dv.ctypes.data, 2, None, arrs, 1, ctypes.byref(nout)) == 28
    assert nout.value == 1

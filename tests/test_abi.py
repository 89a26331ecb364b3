"""The drop-in boundary on CPU: libdk_rx.so loads, exports every function include/*.h declares, the ctypes mirror
matches the C layout, and the verdict/errno tables match the reference's errno per check. No compute calls."""
import ctypes
import os
import re
import subprocess

import pytest

from demikernel_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("dk_rx.h", "dk_diag.h", "dk_ring.h", "dk_tcp.h")]


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
            "dk_tcp_rx_process"} <= names
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert names <= exported, names - exported
    bound = {f[0] for f in N.FUNCTIONS + N.RING_FUNCTIONS + N.TCP_FUNCTIONS + N.DIAG_FUNCTIONS}
    assert bound == names, (names ^ bound)
    for n in names:
        getattr(lib, n)


def test_struct_layout_matches_ctypes(tmp_path):
    """sizeof/offsetof from the C compiler == the ctypes mirror (dk_rx_cfg, dk_flow, dk_rx_batch, dk_rx_results)."""
    structs = {"dk_rx_cfg": N.DkRxCfg, "dk_flow": N.DkFlow, "dk_rx_batch": N.DkRxBatch, "dk_rx_results": N.DkRxResults,
               "dk_tcp_view": N.DkTcpView, "dk_tcp_conn": N.DkTcpConn, "dk_tcp_out": N.DkTcpOut}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADERS[0]}"', f'#include "{HEADERS[3]}"',
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
    for fname, _ in N.DkTcpConn._fields_:
        assert N.CONN_DTYPE.fields[fname][1] == getattr(N.DkTcpConn, fname).offset, fname


def test_tcp_header_constants():
    hdr = open(HEADERS[3]).read()
    for i, name in enumerate(N.TCP_ACTIONS):
        assert re.search(rf"DK_TCP_{name} = {i}[,\s]", hdr), name
    assert f"DK_TCP_OOO_MAX {N.DK_TCP_OOO_MAX}u" in hdr and f"DK_TCP_DELIV_EXTRA {N.DK_TCP_DELIV_EXTRA}u" in hdr
    for name, v in (("NONE", N.DK_TCP_NONE), ("ESTABLISHED", N.DK_TCP_ESTABLISHED), ("CLOSED", N.DK_TCP_CLOSED)):
        assert re.search(rf"DK_TCP_{name} = {v}", hdr), name


def test_verdict_tables():
    lib = N.load_library()
    assert lib.dk_rx_abi_version() == 2
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

"""Bring `lo` up in the current network namespace (SIOCSIFFLAGS |= IFF_UP), for the live TPACKET_V3 ring tests run
where the process has no CAP_NET_RAW of its own: in a fresh user + network namespace (`unshare -rn`, an ordinary user
on the GPU box) the process is root over that namespace's interfaces, whose `lo` starts down. The image has no `ip`.

    unshare -rn sh -c 'python tools/netns_lo_up.py && python -m pytest tests/test_live_ring.py -v'
"""
import fcntl
import socket
import struct

SIOCGIFFLAGS, SIOCSIFFLAGS, IFF_UP = 0x8913, 0x8914, 0x1

s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
req = struct.pack("16sH14x", b"lo", 0)
flags = struct.unpack("16sH14x", fcntl.ioctl(s, SIOCGIFFLAGS, req))[1]
fcntl.ioctl(s, SIOCSIFFLAGS, struct.pack("16sH14x", b"lo", flags | IFF_UP))
flags = struct.unpack("16sH14x", fcntl.ioctl(s, SIOCGIFFLAGS, req))[1]
print(f"lo flags 0x{flags:x} (up: {bool(flags & IFF_UP)})")
s.close()

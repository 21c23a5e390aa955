"""mgh_rendezvous (include/mg_host.h): the TCP hand-over of the RCCL unique id
that the C++ exchange host (mg_overlap -xchg, csrc/host/mg_xchg.cpp) uses at
world > 1.  CPU only: several ranks as threads of this process (ctypes releases
the GIL during the call), host-name resolution, and the bounded waits."""
import ctypes as C
import os
import socket
import threading
import time

import pytest

from metagenomics_amd import overlap


def _lib():
    L = C.CDLL(overlap.LIB_PATH)
    f = L.mgh_rendezvous
    f.restype = C.c_int
    f.argtypes = [C.c_int, C.c_int, C.c_char_p, C.c_int, C.c_void_p, C.c_uint64, C.c_int]
    return f


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, addr, payload, timeout_ms=20000, skip=()):
    f = _lib()
    port = _free_port()
    bufs = [C.create_string_buffer(payload if r == 0 else b"\0" * len(payload), len(payload)) for r in range(world)]
    rcs = [None] * world

    def go(r):
        rcs[r] = f(r, world, addr.encode(), port, C.cast(bufs[r], C.c_void_p), len(payload), timeout_ms)

    ts = [threading.Thread(target=go, args=(r,)) for r in range(world) if r not in skip]
    # the other ranks start first: they must retry until rank 0 listens
    for t in reversed(ts):
        t.start()
        time.sleep(0.02)
    for t in ts:
        t.join(timeout=timeout_ms / 1000 + 30)
    return rcs, [b.raw for b in bufs]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rendezvous_hands_the_id_to_every_rank(world):
    payload = os.urandom(128)  # sizeof(ncclUniqueId)
    rcs, got = _run(world, "127.0.0.1", payload)
    assert rcs == [0] * world
    assert all(g == payload for g in got)


def test_rendezvous_resolves_host_names():
    payload = os.urandom(128)
    rcs, got = _run(3, "localhost", payload)
    assert rcs == [0, 0, 0] and all(g == payload for g in got)


def test_rendezvous_world_one_is_a_no_op():
    f = _lib()
    buf = C.create_string_buffer(b"x" * 16, 16)
    assert f(0, 1, b"127.0.0.1", 1, C.cast(buf, C.c_void_p), 16, 100) == 0


def test_rendezvous_bad_arguments_and_names():
    f = _lib()
    buf = C.create_string_buffer(16)
    assert f(2, 2, b"127.0.0.1", 1234, C.cast(buf, C.c_void_p), 16, 100) == -1  # rank out of range
    assert f(1, 2, b"no-such-host.invalid", _free_port(), C.cast(buf, C.c_void_p), 16, 2000) == -2


def test_rendezvous_missing_peer_times_out():
    # rank 1 of 3 never starts: rank 0 gives up at its deadline instead of hanging in accept()
    t0 = time.time()
    rcs, _ = _run(3, "127.0.0.1", os.urandom(32), timeout_ms=1500, skip=(1,))
    assert rcs[0] == -4 and rcs[1] is None
    assert rcs[2] in (0, -5)  # it may or may not have been served before rank 0 gave up
    assert time.time() - t0 < 20


def test_rendezvous_missing_rank0_times_out():
    rcs, _ = _run(2, "127.0.0.1", os.urandom(32), timeout_ms=1000, skip=(0,))
    assert rcs[1] == -4


def _strays(port, stop, kinds):
    """Connections to rank 0's port that are not ranks: silent, garbage, a duplicate rank."""
    import struct

    socks = []
    while not stop.is_set() and len(socks) < len(kinds):
        k = kinds[len(socks)]
        try:
            s = socket.create_connection(("127.0.0.1", port), timeout=0.2)
        except OSError:
            time.sleep(0.02)
            continue
        if k == "garbage":
            s.sendall(b"GET / HTTP/1.0\r\n\r\n")
        elif k == "dup":
            s.sendall(struct.pack("<II", 0x4D47525A, 1))
        elif k == "rank0":
            s.sendall(struct.pack("<II", 0x4D47525A, 0))
        socks.append(s)
    stop.wait(10)
    for s in socks:
        s.close()


@pytest.mark.parametrize("kinds", [("silent",), ("garbage", "rank0"), ("dup", "silent", "garbage")])
def test_rendezvous_ignores_stray_connections(kinds):
    """A port probe or a health check that connects before the ranks does not use
    up a rank's place (rank 0 checks each peer's header and serves every rank once)."""
    f = _lib()
    world, payload = 3, os.urandom(128)
    port = _free_port()
    bufs = [C.create_string_buffer(payload if r == 0 else b"\0" * len(payload), len(payload)) for r in range(world)]
    rcs = [None] * world
    stop = threading.Event()

    def go(r):
        rcs[r] = f(r, world, b"127.0.0.1", port, C.cast(bufs[r], C.c_void_p), len(payload), 20000)

    t0 = threading.Thread(target=go, args=(0,))
    t0.start()
    ts = threading.Thread(target=_strays, args=(port, stop, kinds))
    ts.start()
    time.sleep(0.5)  # the strays reach rank 0 first
    peers = [threading.Thread(target=go, args=(r,)) for r in range(1, world)]
    for t in peers:
        t.start()
    for t in [t0] + peers:
        t.join(60)
    stop.set()
    ts.join(30)
    if "dup" in kinds:  # the duplicate may have taken rank 1's place before it came: then rank 1 is refused
        assert rcs[0] == 0 and rcs[2] == 0 and rcs[1] in (0, -5)
        assert bufs[2].raw == payload
    else:
        assert rcs == [0] * world
        assert all(b.raw == payload for b in bufs)

"""End to end through the daemon on the GPU: frames enter over the NIC wire,
the kernel host ring and two RequestUDS clients, are classified by the HIP
path in poll-round batches, and must come out of exactly the sockets the
sequential oracle's decisions name (Target::Endpoint/Nic/Last, mirror_to_all
for FLOOD, nothing for None), in order.
"""
import os
import random
import socket
import time

import pytest

import randtraffic
from daemon_client import Daemon, want

pytestmark = pytest.mark.gpu

MACS = ["02:00:00:00:00:03", "02:00:00:00:00:04"]


def _sink(path):
    s = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
    s.bind(path)
    s.setblocking(False)
    return s


def _drain(sock, into, deadline):
    while time.time() < deadline:
        try:
            into.append(sock.recv(65536))
        except BlockingIOError:
            time.sleep(0.002)
            if not sock_has_more(sock):
                return


def sock_has_more(sock):
    import select
    r, _, _ = select.select([sock], [], [], 0.05)
    return bool(r)


def _pcap_frames(path):
    """Frames of a libpcap file (Ethernet, the reference's PcapSink format)."""
    import struct
    data = open(path, "rb").read()
    magic, _, _, _, _, snap, link = struct.unpack("<IHHiIII", data[:24])
    assert magic == 0xA1B2C3D4 and link == 1
    out, at = [], 24
    while at + 16 <= len(data):
        _, _, incl, orig = struct.unpack("<IIII", data[at:at + 16])
        out.append(data[at + 16:at + 16 + incl])
        assert incl == orig
        at += 16 + incl
    assert at == len(data)
    return out


def _subsequence(seq, of):
    it = iter(of)
    return all(any(x == y for y in it) for x in seq)


@pytest.mark.parametrize("devices", [None, "0,0"], ids=["one-gpu", "two-replicas"])
def test_daemon_forwards_like_the_oracle(devices, tmp_path):
    """...and PCAP_LOG (src/main.rs:635-648, hook src/endpoint.rs:47-52) holds
    every received frame, each source's in its order.  "two-replicas": the
    daemon over USNETD_HIP_DEVICES=0,0 (one registry, two device copies of the
    rule image; the NIC on one, nothing changes in what comes out)."""
    import coracle
    coracle.build()
    envs = {"INTERFACES": "eth0", "ADD_MACS": ",".join(MACS), "USNETD_MAX_BATCH": "64",
            "USNETD_WRITE_WAIT_MS": "5000", "PCAP_LOG": str(tmp_path / "rx.pcap")}
    if devices:
        envs["USNETD_HIP_DEVICES"] = devices
    d = Daemon(envs, control_only=False)
    bursts = []
    try:
        assert d.p.poll() is None, d.log_text()
        wire = _sink(os.path.join(d.dir, "eth0.wire"))
        kernel = _sink(os.path.join(d.dir, "eth0.kernel"))
        a, b = d.client("a"), d.client("b")
        assert a.request_uds("eth0")[0] == "$" and b.request_uds("eth0")[0] == "$"
        a.fd.setblocking(False)
        b.fd.setblocking(False)
        o = coracle.Oracle()
        for eid, kind, nic in [(0, 0, -1), (1, 1, 0), (2, 3, 0), (3, 3, 0)]:
            o.add_endpoint(eid, kind, nic)
        for m in MACS:
            o.bridge_add(bytes.fromhex(m.replace(":", "")))
        rules = [(a, 2, want("10.0.0.2", 17, 80)), (a, 2, want("10.0.0.2", 6, 443)),
                 (b, 3, want("10.0.0.3", 17, 9999)), (b, 3, want("10.0.0.4", 6, 22, "10.0.0.2", 80))]
        for c, owner, w in rules:
            assert c.ask({"AddMatch": w}) == "OK"
            o.add_match(coracle.make_want(w["dst_addr"]["Ipv4"], w["protocol"], w["dst_port"],
                                          w["src_addr"] and w["src_addr"]["Ipv4"], w["src_port"]),
                        owner)
        # the daemon's sockets per endpoint id: where a frame for that id comes out
        out = {0: wire, 1: kernel, 2: a.fd, 3: b.fd}
        inj = {0: (wire, os.path.join(d.dir, "eth0.nic")), 1: (kernel, os.path.join(d.dir, "eth0.host")),
               2: (a.fd, None), 3: (b.fd, None)}
        rng = random.Random(7)
        expect = {k: [] for k in out}
        got = {k: [] for k in out}
        for burst in range(24):
            src = rng.choice([0, 0, 0, 1, 2, 3])
            frames = [randtraffic.rand_frame(rng, [1, 2]) for _ in range(rng.randrange(1, 80))]
            bursts.append(frames)
            for f in frames:
                dec = o.forward(src, f)
                cls, ep = (dec >> 16) & 0xF, dec & 0xFFFF
                targets = [] if cls == 0 else [k for k in out if k != src] if cls == 3 else [ep]
                for t in targets:
                    if t in expect:
                        expect[t].append(f)
                s, path = inj[src]
                t_end = time.time() + 10
                while True:   # AF_UNIX datagram queues are short: keep the sinks drained
                    try:
                        if path:
                            s.sendto(f, path)
                        else:
                            s.send(f)
                        break
                    except BlockingIOError:
                        assert time.time() < t_end, "daemon stopped reading"
                        for k2, s2 in out.items():
                            _drain(s2, got[k2], time.time() + 0.01)
            deadline = time.time() + 5
            for k, s in out.items():
                _drain(s, got[k], deadline)
        end = time.time() + 15
        while time.time() < end and any(len(got[k]) < len(expect[k]) for k in out):
            for k, s in out.items():
                _drain(s, got[k], time.time() + 0.5)
        time.sleep(0.2)
        for k, s in out.items():
            _drain(s, got[k], time.time() + 0.2)
        for k in out:
            assert len(got[k]) == len(expect[k]), (k, len(got[k]), len(expect[k]), d.log_text()[-2000:])
            assert got[k] == expect[k], k
        assert sum(len(v) for v in expect.values()) > 100
    finally:
        rc = d.stop()
    assert rc == 0, d.log_text()[-3000:]
    dumped = _pcap_frames(str(tmp_path / "rx.pcap"))
    sent = [f for b in bursts for f in b]
    assert sorted(dumped) == sorted(sent)
    for b in bursts:
        assert _subsequence(b, dumped)

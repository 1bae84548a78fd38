"""The usnetd daemon's control plane on CPU (registry-only context).

Each case restates a branch of act_on (/root/reference/src/main.rs:403-633),
the socket setup (:886-903), the config handling (:818-957), the client
liveness check (:1050-1057) and the timer/cleanup protocol (:673-701,
:1070-1110): the reply the reference sends, or its silence.
"""
import json
import os
import stat
import subprocess
import time

import pytest

from daemon_client import DAEMON, Daemon, want

BASE = {"INTERFACES": "eth0", "DEBUG_PORTS": "eth0:TCP:22", "USNETD_IFACE_IP_eth0": "10.0.0.1",
        "ADD_MACS": "02:00:00:00:00:01,02:00:00:00:00:02"}


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(DAEMON):
        subprocess.run(["make", "-s", "usnetd_amd/bin/usnetd"], check=True,
                       cwd=os.path.dirname(os.path.dirname(DAEMON)) + "/..")
    assert os.path.exists(DAEMON)


@pytest.fixture
def daemon():
    d = Daemon(BASE)
    yield d
    d.stop()


def rules_of(dump):
    return sorted(tuple(r) for r in dump["rules"])


def test_startup_state_and_socket_mode(daemon):
    assert stat.S_IMODE(os.stat(daemon.sock).st_mode) == 0o770
    c = daemon.client()
    d = c.dump()
    kinds = [(e[0], e[1], e[2], e[3]) for e in d["endpoints"]]
    assert kinds == [(0, 0, -1, "eth0"), (1, 1, 0, "eth0")]   # NIC, then its host ring
    # DEBUG_PORTS eth0:TCP:22 -> sticky listening rule of the host ring
    assert rules_of(d) == [(0x0A000001, 0, 22, 0, 6, 1, 1, 1)]
    assert d["bridge"] == 2


def test_request_uds_and_add_match(daemon):
    c = daemon.client("a")
    # AddMatch before the client owns an endpoint: silence (:531-533)
    assert c.ask({"AddMatch": want("10.0.0.1", 17, 5353)}, timeout=0.3) is None
    assert c.ask({"RequestNetmapPipe": ["eth0", 1]}) == "ER"          # built without netmap
    msg, fd = c.request_uds("eth0")
    assert msg == "$" and fd is not None
    d = c.dump()
    assert d["endpoints"][-1][1:5] == [3, 0, "", c.path]
    assert c.ask({"AddMatch": want("10.0.0.1", 17, 5353)}) == "OK"
    assert c.ask({"AddMatch": want("10.0.0.1", 17, 5353)}) == "ER"     # key exists (:272-274)
    b = daemon.client("b")
    assert b.request_uds("eth0")[0] == "$"
    assert b.ask({"AddMatch": want("10.0.0.1", 17, 5353)}) == "ER"
    assert b.ask({"AddMatch": want("10.0.0.1", 6, 8080, "10.0.0.9", 40000)}) == "OK"
    r = rules_of(c.dump())
    own = {x[6] for x in r if x[2] == 5353}
    assert own == {2}
    assert (0x0A000001, 0x0A000009, 8080, 40000, 6, 7, 3, 0) in r
    assert daemon.client("x").request_uds("nope") == ("ER", None)       # NIC not found (:457-465)


def test_query_used_ports(daemon):
    c = daemon.client()
    c.request_uds("eth0")
    c.ask({"AddMatch": want("10.0.0.1", 17, 53)})
    c.ask({"AddMatch": want("10.0.0.1", 6, 443, "192.168.1.7", 51000)})
    c.ask({"AddMatch": want("10.0.0.1", 1)})                     # no port: not listed
    ans = c.ask('"QueryUsedPorts"')
    assert ans.startswith('{"QueryUsedPortsAnswer":{"listening":[') and " " not in ans
    body = json.loads(ans)["QueryUsedPortsAnswer"]
    assert sorted(map(tuple, (tuple([t[0], t[1]["Ipv4"], t[2]]) for t in body["listening"]))) == \
        [(6, "10.0.0.1", 22), (17, "10.0.0.1", 53)]
    assert [tuple([t[0], t[1]["Ipv4"], t[2]]) for t in body["connected"]] == [(6, "10.0.0.1", 443)]
    # any sender may ask, endpoint or not (:549-577)
    assert daemon.client("z").ask({"QueryUsedPorts": None}).startswith('{"QueryUsedPortsAnswer"')


def test_remove_match_owner_check_and_silence(daemon):
    a, b = daemon.client("a"), daemon.client("b")
    a.request_uds("eth0")
    b.request_uds("eth0")
    assert a.ask({"AddMatch": want("10.0.0.1", 17, 7000)}) == "OK"
    assert b.ask({"RemoveMatch": want("10.0.0.1", 17, 7000)}, timeout=0.3) is None
    assert any(r[2] == 7000 for r in a.dump()["rules"])                 # not the owner: kept
    assert a.ask({"RemoveMatch": want("10.0.0.1", 17, 7000)}, timeout=0.3) is None
    assert not any(r[2] == 7000 for r in a.dump()["rules"])
    assert a.ask({"RemoveMatch": want("10.0.0.1", 17, 7000)}, timeout=0.3) is None   # absent


def test_delete_client_drops_endpoint_and_rules(daemon):
    a = daemon.client("a")
    a.request_uds("eth0")
    assert a.ask({"AddMatch": want("10.0.0.1", 17, 9000)}) == "OK"
    a.send('"DeleteClient"')
    time.sleep(0.2)
    d = a.dump()
    assert len(d["endpoints"]) == 2 and not any(r[2] == 9000 for r in d["rules"])
    # the client no longer owns an endpoint: AddMatch is silent again
    assert a.ask({"AddMatch": want("10.0.0.1", 17, 9000)}, timeout=0.3) is None


@pytest.mark.parametrize("msg,reply", [
    # serde shapes of the same AddMatch
    ('{"AddMatch":{"dst_addr":{"Ipv4":"10.0.0.1"},"protocol":17,"dst_port":1001}}', "OK"),
    ('{"AddMatch":[{"Ipv4":"10.0.0.1"},1002,null,null,17]}', "OK"),
    ('{"AddMatch":{"dst_addr":{"Ipv4":"10.0.0.1"},"dst_port":1003,"src_addr":null,'
     '"src_port":null,"protocol":17,"extra":[1,2]}}', "OK"),
    (' {"AddMatch" : {"dst_addr":{"Ipv4":"010.000.000.001"},"dst_port":1004,"protocol":17}}\n', "OK"),
    # rejected by serde / Ipv4Address::from_str: silence
    ('{"AddMatch":{"dst_addr":{"Ipv4":"10.0.0.1"},"dst_port":1005}}', None),
    ('{"AddMatch":{"dst_addr":{"Ipv4":"10.0.0.1"},"dst_port":1006,"protocol":256}}', None),
    ('{"AddMatch":{"dst_addr":{"Ipv4":"10.0.0.1"},"dst_port":65536,"protocol":17}}', None),
    ('{"AddMatch":{"dst_addr":{"Ipv4":"10.0.0.1"},"dst_port":1008.0,"protocol":17}}', None),
    ('{"AddMatch":{"dst_addr":{"Ipv4":"10.0.0.1"},"protocol":17,"protocol":6}}', None),
    ('{"AddMatch":{"dst_addr":{"Ipv4":"10.0.0.256"},"dst_port":1010,"protocol":17}}', None),
    ('{"AddMatch":{"dst_addr":{"Ipv4":"10.0.0.1 "},"dst_port":1011,"protocol":17}}', None),
    ('{"AddMatch":{"dst_addr":{"Ipv6":"::1"},"dst_port":1012,"protocol":17}}', None),
    ('{"AddMatch":[{"Ipv4":"10.0.0.1"},1013,null,null]}', None),
    ('{"AddMatch":{"dst_addr":"10.0.0.1","dst_port":1014,"protocol":17}}', None),
    ('{"AddMatch":{"dst_addr":{"Ipv4":"10.0.0.1"},"dst_port":1015,"protocol":17},}', None),
    ('{"AddMatch":{"dst_addr":{"Ipv4":"10.0.0.1"},"dst_port":1016,"protocol":17}} x', None),
    ('"AddMatch"', None),
    ('{"AddMatch":{"dst_addr":{"Ipv4":"10.0.0.1"},"dst_port":1017,"protocol":17},"QueryUsedPorts":null}', None),
    ('{"Bogus":null}', None),
    ('not json', None),
])
def test_serde_acceptance(daemon, msg, reply):
    c = daemon.client()
    c.request_uds("eth0")
    assert c.ask(msg, timeout=0.3 if reply is None else 2.0) == reply
    assert daemon.p.poll() is None


def test_invalid_src_addr_becomes_none(daemon):
    """new_from_want_msg: an unparsable src_addr is .ok() -> None (pkt.rs:242-247)."""
    c = daemon.client()
    c.request_uds("eth0")
    assert c.ask({"AddMatch": want("10.0.0.1", 6, 2222, "bad", None)}) == "OK"
    assert (0x0A000001, 0, 2222, 0, 6, 1, 2, 0) in rules_of(c.dump())


def test_datagram_longer_than_4000_bytes_is_not_json(daemon):
    c = daemon.client()
    c.request_uds("eth0")
    msg = '{"AddMatch":' + " " * 4000 + json.dumps(want("10.0.0.1", 17, 1234)) + "}"
    assert c.ask(msg, timeout=0.3) is None


def test_dead_client_pid_is_reaped_on_next_change(daemon):
    p = subprocess.Popen(["true"])
    p.wait()
    a = daemon.client("a")
    a.request_uds("eth0", pid=p.pid)          # pid already gone
    assert len(a.dump()["endpoints"]) == 3    # checked only when some change happens
    b = daemon.client("b")
    b.request_uds("eth0")                      # a change: liveness is probed (:1050-1057)
    time.sleep(0.1)
    eps = b.dump()["endpoints"]
    assert [e[4] for e in eps] == ["", "", b.path]


def test_cleanup_keeps_sticky_and_end_stops():
    d = Daemon(BASE, cleanup_secs=1)
    try:
        c = d.client()
        time.sleep(2.5)                         # at least one timer "cleanup"
        assert rules_of(c.dump()) == [(0x0A000001, 0, 22, 0, 6, 1, 1, 1)]
        c.send("end")
        assert d.p.wait(5) == 0
    finally:
        d.stop()
    assert "cleanup" in d.log_text()


def test_sigterm_clean_shutdown():
    d = Daemon(BASE)
    t0 = time.time()
    assert d.stop() == 0 and time.time() - t0 < 5
    assert not os.path.exists(d.sock)


@pytest.mark.parametrize("env,ok", [
    ({"INTERFACES": "eth0", "NO_HOST_RINGS": "true"}, True),
    ({}, False),                                                    # INTERFACES required
    ({"INTERFACES": "eth0", "STATIC_PIPES": "eth0:UDP:53"}, False),   # needs netmap
    ({"INTERFACES": "eth0", "NO_HOST_RINGS": "true", "DEBUG_PORTS": "eth0:TCP:22",
      "USNETD_IFACE_IP_eth0": "10.0.0.1"}, False),                  # host ring not found
    ({"INTERFACES": "eth0", "DEBUG_PORTS": "eth0:SCTP:9"}, False),
])
def test_config_errors(env, ok):
    e = {"INTERFACES": ""}
    e.update(env)
    if "INTERFACES" not in env:
        e = {k: v for k, v in e.items() if k != "INTERFACES"}
        saved = os.environ.pop("INTERFACES", None)
    d = Daemon(e)
    try:
        if ok:
            assert d.p.poll() is None
            assert [x[1] for x in d.client().dump()["endpoints"]] == [0]
        else:
            assert d.p.wait(5) == 1
    finally:
        d.stop()
        if "INTERFACES" not in env and saved is not None:
            os.environ["INTERFACES"] = saved


def test_conffile_is_fallback(tmp_path):
    conf = tmp_path / "usnetd.conf"
    conf.write_text("# comment\nINTERFACES=eth7\nNO_HOST_RINGS=true\nRUST_LOG=debug\n")
    import tempfile
    sdir = tempfile.mkdtemp()
    sock = os.path.join(sdir, "usnetd.socket")
    e = dict(os.environ, USNETD_SOCKET=sock, USNETD_CONTROL_ONLY="1", USNETD_TEST_DUMP="1")
    e.pop("INTERFACES", None)
    p = subprocess.Popen([DAEMON, str(conf)], env=e, stderr=subprocess.PIPE)
    try:
        for _ in range(100):
            if os.path.exists(sock):
                break
            time.sleep(0.02)
        import socket as S
        s = S.socket(S.AF_UNIX, S.SOCK_DGRAM)
        s.bind(os.path.join(sdir, "c"))
        s.settimeout(2)
        s.sendto(b"dump", sock)
        eps = json.loads(s.recv(65536))["endpoints"]
        assert [(x[1], x[3]) for x in eps] == [(0, "eth7")]
    finally:
        p.terminate()
        p.wait(5)

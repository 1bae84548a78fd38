"""Helpers to run the usnetd daemon binary and talk to its control socket."""
from __future__ import annotations

import array
import json
import os
import socket
import subprocess
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DAEMON = os.path.join(ROOT, "usnetd_amd", "bin", "usnetd")


class Daemon:
    """Starts `usnetd` with a private socket directory."""

    def __init__(self, env: dict, control_only=True, cleanup_secs=3600):
        self.dir = tempfile.mkdtemp(prefix="usnd")
        self.sock = os.path.join(self.dir, "usnetd.socket")
        e = dict(os.environ)
        e.update({"USNETD_SOCKET": self.sock, "USNETD_TEST_DUMP": "1",
                  "USNETD_CLEANUP_SECS": str(cleanup_secs), "RUST_LOG": "info"})
        if control_only:
            e["USNETD_CONTROL_ONLY"] = "1"
        e.update(env)
        self.log = open(os.path.join(self.dir, "daemon.log"), "w")
        self.p = subprocess.Popen([DAEMON], env=e, stdout=self.log, stderr=subprocess.STDOUT)
        for _ in range(200):
            if os.path.exists(self.sock) or self.p.poll() is not None:
                break
            time.sleep(0.02)
        time.sleep(0.05)

    def client(self, name="c") -> "Client":
        return Client(self, name)

    def stop(self, timeout=10):
        if self.p.poll() is None:
            self.p.terminate()   # SIGTERM -> the timer thread sends "end"
            try:
                self.p.wait(timeout)
            except subprocess.TimeoutExpired:
                self.p.kill()
                self.p.wait()
        self.log.close()
        return self.p.returncode

    def log_text(self):
        with open(os.path.join(self.dir, "daemon.log")) as fh:
            return fh.read()


class Client:
    """A control-socket client bound to its own path (client_path)."""

    def __init__(self, d: Daemon, name: str):
        self.d = d
        self.path = os.path.join(d.dir, "client-" + name)
        self.s = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
        self.s.bind(self.path)
        self.s.settimeout(2.0)
        self.fd = None

    def send(self, msg):
        data = msg if isinstance(msg, (bytes, str)) else json.dumps(msg)
        if isinstance(data, str):
            data = data.encode()
        self.s.sendto(data, self.d.sock)

    def recv(self, timeout=2.0):
        self.s.settimeout(timeout)
        try:
            return self.s.recv(65536).decode()
        except socket.timeout:
            return None

    def ask(self, msg, timeout=2.0):
        self.send(msg)
        return self.recv(timeout)

    def request_uds(self, iface, pid=None):
        """RequestUDS -> ("$", fd) or ("ER", None)."""
        self.send({"RequestUDS": [iface, os.getpid() if pid is None else pid]})
        fds = array.array("i")
        msg, anc, _, _ = self.s.recvmsg(64, socket.CMSG_LEN(fds.itemsize))
        for level, typ, data in anc:
            if level == socket.SOL_SOCKET and typ == socket.SCM_RIGHTS:
                fds.frombytes(data[:len(data) - (len(data) % fds.itemsize)])
        fd = fds[0] if len(fds) else None
        if fd is not None:
            self.fd = socket.socket(fileno=fd)
        return msg.decode(), fd

    def dump(self):
        return json.loads(self.ask("dump"))

    def close(self):
        self.s.close()
        if self.fd is not None:
            self.fd.close()


def want(dst, proto, dport=None, src=None, sport=None):
    return {"dst_addr": {"Ipv4": dst}, "dst_port": dport,
            "src_addr": None if src is None else {"Ipv4": src}, "src_port": sport, "protocol": proto}

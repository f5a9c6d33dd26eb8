"""Process harness for the master/worker plumbing tests: starts a master (the build's
dsort_master or the reference's server) and N workers (the build's dsort_worker or the
reference's client) on 127.0.0.1, feeds file names on the master's stdin and collects
output.txt.  Used by tests/test_plumbing.py (CPU, with the C-ABI test double) and
tests/test_gpu_plumbing.py (GPU box, with the real libdsort.so)."""
import os
import socket
import subprocess
import time

from conftest import PKG, REF_BUILD, REPO

BIN = os.path.join(PKG, "bin")
DOUBLE_DIR = os.path.join(REPO, "tests", "double")
DOUBLE_LIB_DIR = os.path.join(DOUBLE_DIR, "build")


def build_double():
    """Builds the CPU test double of libdsort (tests/double/dsort_double.c + the oracle)."""
    os.makedirs(DOUBLE_LIB_DIR, exist_ok=True)
    out = os.path.join(DOUBLE_LIB_DIR, "libdsort.so")
    srcs = [os.path.join(DOUBLE_DIR, "dsort_double.c"), os.path.join(REPO, "oracle", "oracle.c")]
    if not os.path.exists(out) or any(os.path.getmtime(s) > os.path.getmtime(out) for s in srcs):
        subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", out, *srcs])
    return DOUBLE_LIB_DIR


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def established(port):
    """Number of accepted-or-pending TCP connections whose local port is `port` (the master's
    side), in any state but LISTEN: a worker that already died still counts (CLOSE_WAIT)."""
    n = 0
    for path in ("/proc/net/tcp", "/proc/net/tcp6"):
        try:
            with open(path) as f:
                next(f)
                for line in f:
                    parts = line.split()
                    if parts[3] != "0A" and int(parts[1].split(":")[1], 16) == port:
                        n += 1
        except OSError:
            pass
    return n


def listening(port):
    """True once some socket LISTENs on `port` (read from /proc, without connecting: a probe
    connection would take one of the master's accept() slots)."""
    for path in ("/proc/net/tcp", "/proc/net/tcp6"):
        try:
            with open(path) as f:
                next(f)
                for line in f:
                    parts = line.split()
                    if parts[3] == "0A" and int(parts[1].split(":")[1], 16) == port:
                        return True
        except OSError:
            pass
    return False


class Session:
    def __init__(self, workdir, workers=4, master="ours", worker_kinds=None, worker_args=None,
                 master_args=(), lib_dir=None, proto="v0", bin_dir=BIN, env=None):
        self.dir = str(workdir)
        self.n = workers
        self.env = dict(os.environ if env is None else env)
        if lib_dir:
            self.env["LD_LIBRARY_PATH"] = lib_dir + ":" + self.env.get("LD_LIBRARY_PATH", "")
        if master == "ours":
            cmd = [os.path.join(bin_dir, "dsort_master"), "--workers", str(workers), "--proto", proto,
                   *master_args, "server.conf"]
        else:
            cmd = [os.path.join(REF_BUILD, "server"), "server.conf"]
        # free_port() can lose its port to another process before the master binds it (seen on a
        # shared GPU box): a master that exits with "Address already in use" is restarted on a
        # fresh port, up to 5 times
        for attempt in range(5):
            self.port = free_port()
            with open(os.path.join(self.dir, "server.conf"), "w") as f:
                f.write(f"SERVER_PORT={self.port}\n")
            with open(os.path.join(self.dir, "client.conf"), "w") as f:
                f.write(f"SERVER_IP=127.0.0.1\nSERVER_PORT={self.port}\n")
            self.mlog = open(os.path.join(self.dir, "master.log"), "w")
            self.master = subprocess.Popen(cmd, cwd=self.dir, stdin=subprocess.PIPE, stdout=self.mlog,
                                           stderr=subprocess.STDOUT, env=self.env)
            t0 = time.time()
            while not listening(self.port):
                if self.master.poll() is not None or time.time() - t0 > 30:
                    break
                time.sleep(0.02)
            else:
                break
            log = self.master_log()
            if self.master.poll() is None or "Address already in use" not in log or attempt == 4:
                raise RuntimeError("master did not start: " + log)
            self.mlog.close()
        kinds = worker_kinds or ["ours"] * workers
        wargs = worker_args or [[] for _ in range(workers)]
        self.workers = []
        for i, kind in enumerate(kinds):
            log = open(os.path.join(self.dir, f"worker{i + 1}.log"), "w")
            if kind == "ours":
                wc = [os.path.join(bin_dir, "dsort_worker"), "--proto", proto, *wargs[i], "client.conf"]
            else:
                wc = [os.path.join(REF_BUILD, "client"), "client.conf"]
            p = subprocess.Popen(wc, cwd=self.dir, stdout=log, stderr=subprocess.STDOUT, env=self.env)
            self.workers.append(p)
            # accept order = worker identity (server.c:148): wait for this worker's connection
            # before starting the next (a GPU worker connects only after its context is up)
            t0 = time.time()
            while established(self.port) < i + 1 and p.poll() is None and time.time() - t0 < 60:
                time.sleep(0.01)

    def sort_files(self, names, timeout=120):
        self.master.stdin.write(("\n".join(names) + "\nexit\n").encode())
        self.master.stdin.flush()
        self.master.stdin.close()
        try:
            self.master.wait(timeout=timeout)
        finally:
            self.close()
        return self.master.returncode

    def close(self):
        for w in self.workers:
            try:
                w.wait(timeout=10)
            except subprocess.TimeoutExpired:
                w.kill()
                w.wait()
        if self.master.poll() is None:
            self.master.kill()
            self.master.wait()
        self.mlog.close()

    def master_log(self):
        if not self.mlog.closed:
            self.mlog.flush()
        return open(os.path.join(self.dir, "master.log")).read()

    def output(self, name="output.txt"):
        with open(os.path.join(self.dir, name), "rb") as f:
            return f.read()

"""Multi-process launcher: one process per rank on one node (replaces docker compose).

The reference starts every rank in its own container (``codes/task2/docker-compose.yml``:
two GPU services ``node01``/``node02`` running ``model.py --n_devices=2 --rank=r
--master_addr=node01``; ``codes/task4/docker-compose.yml``: three CPU services, the
workers ``depends_on: node01``), or by hand in several terminals (``task2.tex:86-93``).
On an 8x MI355X node the ranks are plain processes: one per GPU, rendezvous over
env:// at 127.0.0.1, RCCL over xGMI once the group is up.

    python -m dmlab.launch --nproc 8 -m dmlab.tasks.task3 --epochs 1
    python -m dmlab.launch --nproc 2 --cpu -- dmlab/tasks/task2.py --aggregation allgather
    python -m dmlab.launch --config configs/task4_rpc.yaml

Every rank gets ``RANK WORLD_SIZE LOCAL_RANK LOCAL_WORLD_SIZE MASTER_ADDR
MASTER_PORT`` (torchrun's contract, which ``dmlab.parallel.env.init`` reads; the
device is ``cuda:LOCAL_RANK``, fixing the reference's every-rank-on-GPU-0).
Arguments may contain ``{rank} {world_size} {master_addr} {master_port}``, which
reproduces the reference's per-rank CLI.  Output lines are prefixed with the rank.
Fail-fast: when a rank exits non-zero the others are terminated (SIGTERM, then
SIGKILL after a grace period) and the launcher exits with that rank's code; a global
``--timeout`` bounds the whole job.  Ranks are started as child processes (never
``exec``), each in its own process group so a hung rank and its children can be
killed as a unit.

Config files (YAML, compose-like)::

    master_port: auto            # or a number
    services:                    # one rank per service, in order (rank 0 first)
      node01: {command: [python, -u, -m, dmlab.tasks.task4, --n_devices={world_size}, --rank={rank}]}
      node02: {command: [...], depends_on: [node01], env: {FOO: "1"}}
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import threading
import time

import yaml


def free_port(addr: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def _order(services: dict) -> list[str]:
    """Ranks follow the file order; ``depends_on`` only constrains start order."""
    names = list(services)
    started, out = set(), []

    def visit(n, stack=()):
        if n in started:
            return
        if n in stack:
            raise ValueError(f"dependency cycle through {n}")
        for d in services[n].get("depends_on", []) or []:
            if d not in services:
                raise ValueError(f"{n} depends on unknown service {d}")
            visit(d, stack + (n,))
        started.add(n)
        out.append(n)

    for n in names:
        visit(n)
    return out


class Job:
    def __init__(self, cmds: list[list[str]], envs: list[dict], start_order: list[int] | None = None,
                 prefix: bool = True, grace_s: float = 10.0, out=None):
        self.cmds, self.envs = cmds, envs
        self.order = start_order or list(range(len(cmds)))
        self.prefix, self.grace = prefix, grace_s
        self.out = out or sys.stdout
        self.procs: list[subprocess.Popen | None] = [None] * len(cmds)
        self._lock = threading.Lock()
        self._pumps = []

    def _pump(self, r, stream):
        for line in iter(stream.readline, ""):
            with self._lock:
                self.out.write(f"[rank {r}] {line}" if self.prefix else line)
                self.out.flush()
        stream.close()

    def start(self):
        for r in self.order:
            p = subprocess.Popen(self.cmds[r], env=self.envs[r], stdout=subprocess.PIPE,
                                 stderr=subprocess.STDOUT, text=True, bufsize=1,
                                 start_new_session=True)
            self.procs[r] = p
            t = threading.Thread(target=self._pump, args=(r, p.stdout), daemon=True)
            t.start()
            self._pumps.append(t)

    def _signal_all(self, sig):
        for p in self.procs:
            if p is not None and p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    pass

    def terminate(self):
        self._signal_all(signal.SIGTERM)
        t0 = time.time()
        while time.time() - t0 < self.grace and any(p.poll() is None for p in self.procs if p):
            time.sleep(0.05)
        self._signal_all(signal.SIGKILL)
        for p in self.procs:
            if p is not None:
                p.wait()

    def wait(self, timeout_s: float | None = None) -> int:
        """Exit code of the job: 0 if every rank succeeded, else the first failure's code
        (124 on timeout)."""
        t0 = time.time()
        code = 0
        try:
            while True:
                states = [p.poll() for p in self.procs]
                bad = [(r, c) for r, c in enumerate(states) if c not in (None, 0)]
                if bad:
                    r, code = bad[0]
                    self.out.write(f"[launch] rank {r} exited with {code}; stopping the job\n")
                    break
                if all(c == 0 for c in states):
                    break
                if timeout_s is not None and time.time() - t0 > timeout_s:
                    self.out.write(f"[launch] timeout after {timeout_s:.0f} s; stopping the job\n")
                    code = 124
                    break
                time.sleep(0.05)
        except KeyboardInterrupt:
            code = 130
        if code != 0:
            self.terminate()
        for t in self._pumps:
            t.join(timeout=5)
        self.out.flush()
        return code if code >= 0 else 128 - code


def build(nproc: int, argv: list[str], master_addr: str, master_port: int, cpu: bool,
          extra_env: list[dict] | None = None, module: str | None = None):
    cmds, envs = [], []
    base = dict(os.environ)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL / tensor sharing)
    for r in range(nproc):
        fmt = dict(rank=r, world_size=nproc, master_addr=master_addr, master_port=master_port)
        args = [a.format(**fmt) for a in argv]
        if module:
            cmd = [sys.executable, "-u", "-m", module] + args
        elif args and args[0].endswith(".py"):
            cmd = [sys.executable, "-u"] + args
        else:
            cmd = args
        env = dict(base)
        env.update(RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(nproc), MASTER_ADDR=master_addr,
                   MASTER_PORT=str(master_port), PYTHONUNBUFFERED="1")
        if cpu:
            env["DMLAB_DEVICE"] = "cpu"
            env["OMP_NUM_THREADS"] = str(max(1, (os.cpu_count() or 1) // nproc))
        if extra_env and extra_env[r]:
            env.update({k: str(v) for k, v in extra_env[r].items()})
        cmds.append(cmd)
        envs.append(env)
    return cmds, envs


def from_config(path: str, master_addr: str, cpu: bool):
    with open(path) as f:
        cfg = yaml.safe_load(f)
    services = cfg["services"]
    names = list(services)
    port = cfg.get("master_port", "auto")
    port = free_port(master_addr) if port in (None, "auto") else int(port)
    n = len(names)
    cmds, envs = [], []
    for r, name in enumerate(names):
        svc = services[name]
        c, e = build(n, [str(a) for a in svc["command"]], master_addr, port,
                     cpu or bool(svc.get("cpu", False)), [svc.get("env")] * n)
        cmds.append(c[r])
        envs.append(e[r])
    order = [names.index(s) for s in _order(services)]
    return cmds, envs, order


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--nproc", "--nproc-per-node", type=int, default=1)
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", default="auto")
    ap.add_argument("--cpu", action="store_true", help="CPU ranks (gloo); cores split evenly")
    ap.add_argument("--config", help="compose-like YAML (one service per rank)")
    ap.add_argument("--timeout", type=float, default=None, help="seconds for the whole job")
    ap.add_argument("--no-prefix", action="store_true")
    ap.add_argument("-m", dest="module", help="run a module (python -m) on every rank")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    argv = list(sys.argv[1:] if argv is None else argv)
    # everything after `-m MODULE` (or after `--`) belongs to the ranks' command line
    tail, module = [], None
    for i, t in enumerate(argv):
        if t == "--":
            argv, tail = argv[:i], argv[i + 1:]
            break
        if t == "-m" and i + 1 < len(argv):
            argv, module, tail = argv[:i], argv[i + 1], argv[i + 2:]
            break
    a = ap.parse_args(argv)
    a.module = module or a.module
    cmd = tail + a.cmd
    if a.config:
        cmds, envs, order = from_config(a.config, a.master_addr, a.cpu)
    else:
        if not cmd and not a.module:
            ap.error("nothing to run")
        port = free_port(a.master_addr) if a.master_port == "auto" else int(a.master_port)
        cmds, envs = build(a.nproc, cmd, a.master_addr, port, a.cpu, module=a.module)
        order = None
    job = Job(cmds, envs, order, prefix=not a.no_prefix)
    job.start()
    return job.wait(a.timeout)


if __name__ == "__main__":
    sys.exit(main())

"""Parameter-server job supervisor: launch 1..k PS + N workers, restart on failure.

The reference's ``MonitoredTrainingSession`` survives a PS restart: on
``AbortedError`` / ``UnavailableError`` it recreates the session and the PS
restores from the latest checkpoint (``/root/reference/main.py:140-146`` [TF1-lib]).
Two levels of recovery here:

* **a parameter server dies** (default ``--recover_ps``): only that process is
  relaunched, on the same ports; it restores its shard from the latest checkpoint
  and opens the next session generation, and the workers and the other PS tasks
  rejoin it IN PLACE (``parallel/ps.py`` "Session recovery") -- no worker restarts;
* **a worker dies** (or a PS restart fails, or ``--recover_ps 0``): the attempt is
  torn down and the job restarts as a whole from the last checkpoint -- the same
  recovery torchrun's elastic agent gives the data-parallel mode (``--max-restarts``).

This module is that agent for PS mode:

    python -m distributed_tensorflow_ibm_mnist_amd.parallel.supervisor \\
        --num_ps 1 --num_workers 7 --max_restarts 3 -- --model=lenet5 --train_dir=/tmp/ps ...

* every process gets ``--job_name/--task_id/--ps_hosts/--worker_hosts`` on
  127.0.0.1, fresh ports per attempt (no TIME_WAIT collisions with the dead one);
* the first non-zero exit tears the attempt down (SIGTERM, then SIGKILL after a
  grace period, whole process groups) and starts the next attempt;
* ``TORCHELASTIC_RESTART_COUNT`` carries the attempt number, so fault injection
  (``MNIST_FI_*``, train/hooks.py) fires on attempt 0 only, as under torchrun;
* the PS restores its shard from ``--train_dir`` (``ps.py``), so an attempt
  resumes at the last checkpointed global step and applies only the missing
  updates.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence, Tuple

EXIT_FATAL = 86      # parallel/ps.py EXIT_FATAL (kept import-free: the supervisor never loads torch)
EXIT_NO_INPLACE = 87  # parallel/cluster.py: a restarted PS found a finished worker -> whole-job restart

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def free_ports(n: int) -> List[int]:
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


class Attempt:
    def __init__(self, procs: Dict[str, subprocess.Popen], spawn=None):
        self.procs = procs
        self.spawn = spawn                 # spawn(name, env_extra) -> Popen: relaunch one process

    def respawn(self, name: str) -> None:
        """Relaunch one process of this attempt (same flags and ports) as a restart."""
        self.procs[name].wait()
        self.procs[name] = self.spawn(name, {"MNISTX_PS_RESTART": "1"})

    def poll(self) -> Tuple[bool, Optional[Tuple[str, int]]]:
        """(all finished, first failure (name, rc) or None)."""
        done = True
        for name, p in self.procs.items():
            rc = p.poll()
            if rc is None:
                done = False
            elif rc != 0:
                return True, (name, rc)
        return done, None

    def teardown(self, grace_s: float = 10.0) -> None:
        for sig in (signal.SIGTERM, signal.SIGKILL):
            for p in self.procs.values():
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, sig)
                    except ProcessLookupError:
                        pass
            t0 = time.time()
            while time.time() - t0 < grace_s and any(p.poll() is None for p in self.procs.values()):
                time.sleep(0.1)
        for p in self.procs.values():
            p.wait()


def launch(main: str, flags: Sequence[str], num_ps: int, num_workers: int, attempt: int, log_dir: Optional[str],
           env_extra: Optional[Dict[str, str]] = None) -> Attempt:
    ports = free_ports(num_ps + num_workers)
    ps_hosts = ",".join(f"127.0.0.1:{p}" for p in ports[:num_ps])
    wk_hosts = ",".join(f"127.0.0.1:{p}" for p in ports[num_ps:])
    env = dict(os.environ, TORCHELASTIC_RESTART_COUNT=str(attempt), PYTHONUNBUFFERED="1", **(env_extra or {}))
    starts: Dict[str, int] = {}

    def spawn(name: str, extra: Optional[Dict[str, str]] = None) -> subprocess.Popen:
        job, i = name.rstrip("0123456789"), int(name.lstrip("pswoker"))
        n = starts[name] = starts.get(name, -1) + 1
        suffix = f"_restart{n}" if n else ""
        out = open(os.path.join(log_dir, f"attempt{attempt}_{name}{suffix}.log"), "w") if log_dir else None
        return subprocess.Popen(
            [sys.executable, main, *flags, f"--job_name={job}", f"--task_id={i}", f"--ps_hosts={ps_hosts}",
             f"--worker_hosts={wk_hosts}"],
            cwd=ROOT, env=dict(env, **(extra or {})), stdout=out, stderr=subprocess.STDOUT if out else None,
            start_new_session=True)

    procs: Dict[str, subprocess.Popen] = {}
    for job, n in (("ps", num_ps), ("worker", num_workers)):
        for i in range(n):
            procs[f"{job}{i}"] = spawn(f"{job}{i}")
    return Attempt(procs, spawn)


def supervise(flags: Sequence[str], num_ps: int = 1, num_workers: int = 2, max_restarts: int = 3,
              main: Optional[str] = None, log_dir: Optional[str] = None, timeout_s: float = 0.0,
              log=print, recover_ps: bool = True) -> int:
    main = main or os.path.join(ROOT, "main.py")
    if log_dir:
        os.makedirs(log_dir, exist_ok=True)
    t_end = time.time() + timeout_s if timeout_s > 0 else None
    for attempt in range(max_restarts + 1):
        log(f"[supervisor] attempt {attempt}: {num_ps} PS + {num_workers} worker(s)")
        att = launch(main, flags, num_ps, num_workers, attempt, log_dir)
        failure = None
        ps_restarts = 0
        while True:
            done, failure = att.poll()
            if failure is not None and failure[1] == EXIT_FATAL:
                # the process stopped on an error no restart would fix (e.g. a rejected push):
                # neither an in-place PS restart nor a whole-job restart
                log(f"[supervisor] {failure[0]} exited with {failure[1]} (fatal); not restarting")
                att.teardown()
                return EXIT_FATAL
            if (failure is not None and recover_ps and failure[0].startswith("ps") and ps_restarts < max_restarts
                    and failure[1] != EXIT_NO_INPLACE):
                # a parameter server died: relaunch just it; workers rejoin in place
                ps_restarts += 1
                log(f"[supervisor] {failure[0]} exited with {failure[1]}; restarting it in place "
                    f"(PS restart {ps_restarts})")
                att.respawn(failure[0])
                continue
            if done:
                break
            if t_end is not None and time.time() > t_end:
                att.teardown()
                log("[supervisor] job timeout")
                return 124
            time.sleep(0.2)
        if failure is None:
            log(f"[supervisor] attempt {attempt} finished")
            return 0
        name, rc = failure
        log(f"[supervisor] {name} exited with {rc}; tearing down attempt {attempt}")
        att.teardown()
    log(f"[supervisor] giving up after {max_restarts} restart(s)")
    return 1


def main(argv: Optional[Sequence[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    flags: List[str] = []
    if "--" in argv:
        k = argv.index("--")
        argv, flags = argv[:k], argv[k + 1:]
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--num_ps", type=int, default=1)
    ap.add_argument("--num_workers", type=int, default=2)
    ap.add_argument("--max_restarts", type=int, default=3)
    ap.add_argument("--log_dir", default="", help="per-process logs (default: inherit stdout)")
    ap.add_argument("--timeout", type=float, default=0.0, help="whole-job wall limit in seconds (0: none)")
    ap.add_argument("--main", default="", help="training entry point (default: the repo's main.py)")
    ap.add_argument("--recover_ps", type=int, default=1,
                    help="1: relaunch a dead PS in place (workers rejoin without restarting); 0: restart the job")
    a = ap.parse_args(argv)
    return supervise(flags, a.num_ps, a.num_workers, a.max_restarts, a.main or None, a.log_dir or None, a.timeout,
                     recover_ps=bool(a.recover_ps))


if __name__ == "__main__":
    sys.exit(main())

"""Lab-4 pipeline benchmark (BASELINE config 4: the task4 2-stage model across 2 ranks).

Runs ``dmlab.tasks.task4 --mode pipeline --bench-json`` for GPipe and 1F1B at 1/4/8
micro-batches and prints one JSON line per run: step ms, per-stage compute ms and the bubble
(fraction of the step a stage is idle), from HIP events on each stage (wall time on the CPU).

    python tools/bench_pipeline.py --device cuda --transport xgmi [--batch 32] [--steps 300]

With one GPU the two ranks share it (gloo process group for the shape handshake and the
barriers; the stage traffic goes over the chosen transport).  The reference runs this model
as three CPU processes over TensorPipe RPC.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda", choices=["cpu", "cuda"])
    ap.add_argument("--transport", default="xgmi", choices=["pg", "xgmi"])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--micro", default="1,4,8")
    ap.add_argument("--schedules", default="gpipe,1f1b")
    ap.add_argument("--out", default=None, help="append the JSON lines to this file")
    ap.add_argument("--graph", action="store_true",
                    help="capture each stage's step in a hipGraph (xgmi transport)")
    ap.add_argument("--cu-partition", action="store_true",
                    help="each stage on its own half of the CUs (one device per stage, emulated)")
    ap.add_argument("--epochs", type=int, default=0,
                    help="epochs of the 60k-sample synthetic set (0: enough for --steps)")
    a = ap.parse_args()
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="2")
    if a.device == "cuda":
        import torch

        if torch.cuda.device_count() < 2:
            env["DMLAB_BACKEND"] = "gloo"  # RCCL rejects two ranks on one GPU
    lines = []
    for sch in a.schedules.split(","):
        for m in (int(v) for v in a.micro.split(",")):
            with tempfile.TemporaryDirectory() as td:
                js = Path(td) / "b.json"
                cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                       "--nproc-per-node=2", "--master-addr=127.0.0.1", f"--master-port={_port()}",
                       "-m", "dmlab.tasks.task4", "--mode", "pipeline", "--device", a.device,
                       "--synthetic", "--schedule", sch, "--micro", str(m), "--batch-size",
                       str(a.batch), "--max-steps", str(a.steps), "--epochs",
                       str(a.epochs or max(1, -(-a.steps * a.batch // 60000) + 1)),
                       "--transport", a.transport if a.device == "cuda" else "pg",
                       "--bench-json", str(js), "--no-test"]
                if a.cu_partition:
                    cmd.append("--cu-partition")
                if a.graph:
                    cmd.append("--graph")
                r = subprocess.run(cmd, cwd=str(ROOT), env=env, capture_output=True, text=True,
                                   timeout=600)
                if r.returncode != 0:
                    print(r.stdout[-2000:], r.stderr[-3000:], file=sys.stderr)
                    sys.exit(r.returncode)
                ranks = [json.loads((Path(td) / f"b.json.rank{k}").read_text()) for k in range(2)]
            row = {"schedule": sch, "n_micro": m, "batch": a.batch, "device": a.device,
                   "transport": ranks[0]["transport"],
                   "cu_partition": ranks[0].get("cu_partition", False),
                   "graph": ranks[0].get("graph", False),
                   "step_ms": max(x["step_ms"] for x in ranks),
                   "samples_per_s": round(a.batch / max(x["step_ms"] for x in ranks) * 1e3, 1),
                   "stage_compute_ms": [x["compute_ms"] for x in ranks],
                   "bubble": [x["bubble"] for x in ranks], "steps_timed": ranks[0]["steps_timed"],
                   "wall_step_ms": max(x.get("wall_step_ms", float("nan")) for x in ranks)}
            print(json.dumps(row), flush=True)
            lines.append(row)
    if a.out:
        with open(a.out, "a") as f:
            for row in lines:
                f.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()

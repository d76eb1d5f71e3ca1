"""Produce the reference labs' graded deliverables with the harness itself.

The reference's grading checklist asks for comparisons, not code
(/root/reference/sections/checking.tex):
  (a) loss curves of the GD / SGD / Adam optimisers              checking.tex:8
  (b) communication cost of two aggregation primitives           checking.tex:20-21
  (c) the effect of a bottleneck (straggler) node                checking.tex:22
      (hook: codes/task2/model-mp.py:47,61-66,79)
  (d) model quality under random sampling vs random partition    checking.tex:15
  (e) model parallelism (RPC stages, pipeline, horizontal split)  checking.tex:14-15

Every number comes from the lab entry points (``dmlab.tasks.task1``..``task4``), launched
as the labs launch them (``torch.distributed.run`` with one rank per process), on the
learnable synthetic MNIST (no dataset download here).  The default device is the CPU with
the gloo backend, so the report reproduces anywhere; ``--device cuda`` runs the same
sweeps on the GPU (RCCL; ranks share one device when only one is present).

    python tools/lab_report.py [--out profiles/labs] [--device cpu] [--only a,b,c,d,e]

Writes ``<out>/<name>.json`` per experiment, ``<out>/*.png`` figures and ``<out>/REPORT.md``.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import socket
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PY = sys.executable


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(threads):
    e = dict(os.environ)
    e["OMP_NUM_THREADS"] = str(threads)
    e["PYTHONPATH"] = str(ROOT) + os.pathsep + e.get("PYTHONPATH", "")
    e.setdefault("MASTER_ADDR", "127.0.0.1")
    # a harder synthetic MNIST than the default (pixel noise 0.7, 10 % random labels: the
    # test accuracy is capped near 91 %), so the comparisons do not all saturate at 100 %
    e.setdefault("DMLAB_SYNTH_NOISE", "0.7")
    e.setdefault("DMLAB_SYNTH_LABEL_NOISE", "0.1")
    if _SHARED_GPU:
        e.setdefault("DMLAB_BACKEND", "gloo")  # RCCL rejects two ranks on one GPU
    return e


_SHARED_GPU = False  # set in main(): --device cuda with fewer GPUs than ranks


def run_task(mod, args, nproc=1, threads=1, timeout=1200):
    """Run ``python -m dmlab.tasks.<mod>`` (via torch.distributed.run when nproc > 1);
    returns (stdout, wall seconds)."""
    if nproc > 1:
        cmd = [PY, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m", f"dmlab.tasks.{mod}"]
    else:
        cmd = [PY, "-m", f"dmlab.tasks.{mod}"]
    t0 = time.perf_counter()
    r = subprocess.run(cmd + list(args), capture_output=True, text=True, timeout=timeout,
                       env=_env(threads), cwd=str(ROOT))
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(f"{mod} {args} failed:\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}")
    return r.stdout, dt


_LOSS = re.compile(r"Device: (\d+) epoch: (\d+), iters:\s+(\d+), loss: ([\d.]+)")
_LOSS1 = re.compile(r"epoch: (\d+), iters:\s+(\d+), loss: ([\d.]+)")
_ACC = re.compile(r"Test set: Accuracy: (\d+)/(\d+)")
_TT = re.compile(r"Training time: ([\d.eE+-]+)")
_CT = re.compile(r"Total communication time: ([\d.eE+-]+)")


def _losses(out, rank=0):
    return [float(m.group(4)) for m in _LOSS.finditer(out) if int(m.group(1)) == rank]


def _acc(out):
    m = _ACC.search(out)
    return int(m.group(1)) / int(m.group(2)) if m else None


def _plot(path, series, xlabel, ylabel, title):
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    fig, ax = plt.subplots(figsize=(6.4, 4.0))
    for name, (xs, ys) in series.items():
        ax.plot(xs, ys, marker="o", ms=3, label=name)
    ax.set_xlabel(xlabel)
    ax.set_ylabel(ylabel)
    ax.set_title(title)
    ax.grid(alpha=0.3)
    ax.legend()
    fig.tight_layout()
    fig.savefig(path, dpi=110)
    plt.close(fig)


def _bars(path, labels, groups, ylabel, title):
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    fig, ax = plt.subplots(figsize=(7.0, 4.0))
    n = len(groups)
    w = 0.8 / max(n, 1)
    for k, (gname, vals) in enumerate(groups.items()):
        ax.bar([i + k * w for i in range(len(labels))], vals, width=w, label=gname)
    ax.set_xticks([i + w * (n - 1) / 2 for i in range(len(labels))])
    ax.set_xticklabels(labels)
    ax.set_ylabel(ylabel)
    ax.set_title(title)
    ax.grid(alpha=0.3, axis="y")
    ax.legend()
    fig.tight_layout()
    fig.savefig(path, dpi=110)
    plt.close(fig)


# ------------------------------------------------------------------------------ (a)
def exp_optimizers(a, out):
    """task1: GD / SGD (momentum .9) / Adam (reference, no bias correction) loss curves
    from the TensorBoard writer's JSONL mirror (tag 'Train Loss')."""
    res = {}
    variants = {"gd": ["--optimizer", "gd"], "sgd": ["--optimizer", "sgd"],
                "adam": ["--optimizer", "adam"],
                "adam (bias-corrected)": ["--optimizer", "adam", "--bias-correction"]}
    for opt, extra in variants.items():
        with tempfile.TemporaryDirectory() as td:
            args = ["--device", a.device, "--synthetic", "--max-steps", str(a.steps1),
                    "--logdir", td + "/", "--seed", "0"] + extra
            o, dt = run_task("task1", args, threads=min(8, os.cpu_count() or 1))
            pts = []
            for f in Path(td).rglob("scalars.jsonl"):
                for line in f.read_text().splitlines():
                    r = json.loads(line)
                    if r["tag"] == "Train Loss":
                        pts.append((r["step"], r["value"]))
            pts.sort()
            res[opt] = {"steps": [p[0] for p in pts], "loss": [p[1] for p in pts],
                        "test_accuracy": _acc(o), "wall_s": round(dt, 2)}
    (out / "a_optimizers.json").write_text(json.dumps(res, indent=1))
    _plot(out / "a_optimizers.png", {k: (v["steps"], v["loss"]) for k, v in res.items()},
          "step (batch 200)", "train loss (mean of 20 iterations)",
          "Lab 1: GD vs SGD vs Adam (LeNet, synthetic MNIST)")
    return res


# ------------------------------------------------------------------------------ (b)
def exp_comm(a, out):
    """task2: all-reduce vs all-gather aggregation, one flat collective vs one per
    parameter (the reference's call pattern), at 2 / 4 / 8 ranks."""
    res = []
    for ws in a.world_sizes:
        for agg in ("allreduce", "allgather"):
            for gran in ("flat", "per_param"):
                with tempfile.TemporaryDirectory() as td:
                    js = Path(td) / "s.json"
                    args = ["--device", a.device, "--synthetic", "--aggregation", agg,
                            "--granularity", gran, "--max-steps", str(a.steps2), "--no-test",
                            "--epochs", "1", "--json", str(js)]
                    o, dt = run_task("task2", args, nproc=ws)
                    s = json.loads(js.read_text())
                res.append({"world_size": ws, "aggregation": agg, "granularity": gran,
                            "steps": s["steps"], "comm_s": s["comm_time"],
                            "train_s": s["train_time"],
                            "comm_ms_per_step": 1e3 * s["comm_time"] / max(s["steps"], 1),
                            "comm_fraction": s["comm_time"] / max(s["train_time"], 1e-9),
                            "samples_per_s": s["samples_per_s"], "final_loss":
                                (s["losses"] or [None])[-1]})
    if a.device == "cuda":
        # the DEVICE communication paths a one-GPU box can run: the one-shot xGMI peer-memory
        # kernel between two ranks sharing the GPU (IPC-mapped buffers, no host staging), and
        # RCCL itself through a 1-rank communicator (every collective issued, no link traffic)
        for path, ws, agg, gran, extra in (
                ("xgmi kernel", 2, "allreduce_xgmi", "flat", []),
                ("rccl 1-rank", 1, "allreduce", "flat", ["--backend", "nccl", "--force-comm"]),
                ("rccl 1-rank", 1, "allreduce", "per_param", ["--backend", "nccl", "--force-comm"]),
                ("rccl 1-rank", 1, "allgather", "flat", ["--backend", "nccl", "--force-comm"]),
                ("rccl 1-rank", 1, "allgather", "per_param", ["--backend", "nccl", "--force-comm"])):
            with tempfile.TemporaryDirectory() as td:
                js = Path(td) / "s.json"
                args = ["--device", "cuda", "--synthetic", "--aggregation", agg, "--granularity",
                        gran, "--max-steps", str(a.steps2), "--no-test", "--epochs", "1",
                        "--json", str(js)] + extra
                o, dt = run_task("task2", args, nproc=ws)
                s = json.loads(js.read_text())
            res.append({"world_size": ws, "aggregation": agg, "granularity": gran, "path": path,
                        "steps": s["steps"], "comm_s": s["comm_time"], "train_s": s["train_time"],
                        "comm_ms_per_step": 1e3 * s["comm_time"] / max(s["steps"], 1),
                        "comm_fraction": s["comm_time"] / max(s["train_time"], 1e-9),
                        "samples_per_s": s["samples_per_s"],
                        "final_loss": (s["losses"] or [None])[-1]})
    (out / "b_comm.json").write_text(json.dumps(res, indent=1))
    res_pg = [r for r in res if "path" not in r]
    labels = [f"ws={w}" for w in a.world_sizes]
    groups = {}
    for agg in ("allreduce", "allgather"):
        for gran in ("flat", "per_param"):
            groups[f"{agg}/{gran}"] = [r["comm_ms_per_step"] for w in a.world_sizes for r in res_pg
                                       if r["world_size"] == w and r["aggregation"] == agg
                                       and r["granularity"] == gran]
    _bars(out / "b_comm.png", labels, groups, "communication ms / step",
          f"Lab 2: gradient aggregation cost (LeNet 51,902 params, {a.device})")
    return res


# ------------------------------------------------------------------------------ (c)
def exp_straggler(a, out):
    """task2: rank 1 delayed after each aggregation (model-mp.py:64-65) by 0 / 20 / 50 ms;
    rank 0's step time and communication time (it waits for the straggler inside the next
    collective)."""
    res = []
    delays = (0, 20, 50)
    # host: time.sleep on the straggler (the reference's hook); device: a spin kernel on its
    # stream, so the delay sits in the GPU queue in front of the collective (GPU only)
    modes = ("host", "device") if a.device == "cuda" else ("host",)
    for mode in modes:
        for d in delays:
            with tempfile.TemporaryDirectory() as td:
                js = Path(td) / "s.json"
                args = ["--device", a.device, "--synthetic", "--max-steps", str(a.steps3),
                        "--no-test", "--epochs", "1", "--json", str(js)]
                if d:
                    args += ["--straggler-rank", "1", "--straggler-delay-ms", str(d),
                             "--straggler-mode", mode]
                o, dt = run_task("task2", args, nproc=2)
                s = json.loads(js.read_text())
            res.append({"delay_ms": d, "mode": mode, "steps": s["steps"],
                        "step_ms": 1e3 * s["train_time"] / max(s["steps"], 1),
                        "comm_ms_per_step": 1e3 * s["comm_time"] / max(s["steps"], 1),
                        "samples_per_s": s["samples_per_s"]})
    (out / "c_straggler.json").write_text(json.dumps(res, indent=1))
    series = {}
    for mode in modes:
        rs = [r for r in res if r["mode"] == mode]
        series[f"step time, {mode} delay"] = (delays, [r["step_ms"] for r in rs])
        series[f"comm time, {mode} delay"] = (delays, [r["comm_ms_per_step"] for r in rs])
    _plot(out / "c_straggler.png", series, "straggler delay on rank 1 (ms per step)",
          "rank-0 ms per step", f"Lab 2: bottleneck node (2 ranks, all-reduce, {a.device})")
    return res


# ------------------------------------------------------------------------------ (d)
def exp_sampling(a, out):
    """task3: random partition (disjoint shards, DistributedSampler semantics) vs random
    sampling (independent per-rank draws, seed = rank) — loss curve and test accuracy."""
    res = {}
    for mode in ("partition", "random"):
        args = ["--device", a.device, "--synthetic", "--sampler", mode, "--max-steps",
                str(a.steps4), "--epochs", "1", "--lr", "0.01"]
        o, dt = run_task("task3", args, nproc=2)
        ls = _losses(o, 0)
        res[mode] = {"loss": ls, "iters": [20 * (i + 1) for i in range(len(ls))],
                     "test_accuracy": _acc(o)}
    (out / "d_sampling.json").write_text(json.dumps(res, indent=1))
    _plot(out / "d_sampling.png", {f"{k} (acc {v['test_accuracy']:.3f})": (v["iters"], v["loss"])
                                   for k, v in res.items()},
          "iteration (2 ranks x batch 32)", "train loss (rank 0)",
          "Lab 3: random partition vs random sampling")
    return res


# ------------------------------------------------------------------------------ (e)
def exp_model_parallel(a, out):
    """task4: the reference RPC stage model (3 processes), the native pipeline (2 stages,
    1F1B with 1 and 4 micro-batches) and the horizontal (tensor-parallel) split.  Same
    seed, data order and optimiser (SGD lr 0.01, momentum 0.9) for every variant, so the
    curves show the three placements compute the same model."""
    runs = [("rpc", ["--mode", "rpc"], 3), ("pipeline m=1", ["--mode", "pipeline", "--micro", "1"], 2),
            ("pipeline m=4", ["--mode", "pipeline", "--micro", "4"], 2),
            ("tp", ["--mode", "tp"], 2)]
    res = {}
    for name, extra, n in runs:
        args = ["--device", a.device, "--synthetic", "--max-steps", str(a.steps5), "--epochs", "1",
                "--momentum", "0.9"]
        o, dt = run_task("task4", args + extra, nproc=n)
        tt = _TT.search(o)
        ls = _losses(o, n - 1 if name.startswith("pipeline") else 0)  # loss lives on the last stage
        steps = a.steps5
        res[name] = {"ranks": n, "loss": ls, "iters": [20 * (i + 1) for i in range(len(ls))],
                     "train_s": float(tt.group(1)) if tt else None,
                     "step_ms": 1e3 * float(tt.group(1)) / steps if tt else None,
                     "test_accuracy": _acc(o)}
    (out / "e_model_parallel.json").write_text(json.dumps(res, indent=1))
    _plot(out / "e_model_parallel.png", {k: (v["iters"], v["loss"]) for k, v in res.items()},
          "iteration (batch 32)", "train loss", "Lab 4: model-parallel variants")
    return res


def write_report(out, R, a):
    L = [f"# Lab deliverables (generated by `tools/lab_report.py`, device {a.device})", "",
         "Data: the learnable synthetic MNIST of `dmlab/data/datasets.py` with pixel noise 0.7 and "
         "10 % random labels (test accuracy capped near 91 %); every run is a lab entry point "
         "(`dmlab.tasks.task1`..`task4`) launched with `torch.distributed.run`, " +
         ("gloo on the CPU." if a.device == "cpu" else
          "all ranks on the box's one MI355X (native HIP kernels; gloo process groups, since RCCL "
          "rejects two ranks on one GPU, so device tensors are staged through the host for the "
          "collectives: the communication times are those of that path, except the device-path rows of (b): the xGMI peer-memory kernel and a 1-rank RCCL communicator)."), ""]
    if "a" in R:
        L += ["## (a) Optimisers: loss curves (checking.tex:8)", "",
              "![](a_optimizers.png)", "", "| optimiser | first loss | last loss | test accuracy |",
              "|---|---|---|---|"]
        for k, v in R["a"].items():
            L.append(f"| {k} | {v['loss'][0]:.3f} | {v['loss'][-1]:.3f} | {v['test_accuracy']:.3f} |")
        L += ["", "Hyper-parameters are the reference's lab-1 defaults (batch 200, lr 5e-4 * sqrt(200) "
              "for GD and Adam, `codes/task1/pytorch/model.py:96-104`; SGD lr 0.01, momentum 0.9). "
              "The reference Adam has no bias correction (`MyOptimizer.py:39-43`): its first "
              "updates are ~3x lr per weight, which on this data kills the ReLU units (loss stuck "
              "at ln 10); the bias-corrected variant (`--bias-correction`) is shown for "
              "comparison.", ""]
    if "b" in R:
        L += ["## (b) Aggregation primitives: communication cost (checking.tex:20-21)", "",
              "![](b_comm.png)", "",
              "| ranks | path | aggregation | granularity | comm ms/step | comm fraction | samples/s |",
              "|---|---|---|---|---|---|---|"]
        for r in R["b"]:
            path = r.get("path", "process group (gloo, host-staged)" if a.device == "cuda"
                         else "process group")
            L.append(f"| {r['world_size']} | {path} | {r['aggregation']} | {r['granularity']} | "
                     f"{r['comm_ms_per_step']:.3f} | {r['comm_fraction']:.2f} | {r['samples_per_s']:.0f} |")
        if a.device == "cuda":
            L += ["", "Device paths on this one-GPU box: `xgmi kernel` = the one-shot peer-memory "
                  "all-reduce (`csrc/comm_xgmi.hip`) between two ranks sharing the GPU through "
                  "IPC-mapped buffers, one kernel per aggregation, timed with HIP events; `rccl "
                  "1-rank` = the same aggregation calls issued to a 1-rank RCCL communicator "
                  "(`task2 --backend nccl --force-comm`): RCCL's launch and synchronisation cost "
                  "per collective without link traffic, i.e. the floor of what the flat and "
                  "per-parameter call patterns pay on xGMI."]
        L.append("")
    if "c" in R:
        L += ["## (c) Bottleneck node (checking.tex:22)", "", "![](c_straggler.png)", "",
              "| delay mode | delay on rank 1 (ms) | rank-0 step ms | rank-0 comm ms/step | samples/s |",
              "|---|---|---|---|---|"]
        for r in R["c"]:
            L.append(f"| {r.get('mode', 'host')} | {r['delay_ms']} | {r['step_ms']:.2f} | "
                     f"{r['comm_ms_per_step']:.2f} | {r['samples_per_s']:.0f} |")
        L.append("")
    if "d" in R:
        L += ["## (d) Data partitioning: random sampling vs random partition (checking.tex:15)", "",
              "![](d_sampling.png)", "", "| sampler | last loss | test accuracy |", "|---|---|---|"]
        for k, v in R["d"].items():
            L.append(f"| {k} | {v['loss'][-1]:.3f} | {v['test_accuracy']:.3f} |")
        L.append("")
    if "e" in R:
        L += ["## (e) Model parallelism (checking.tex:14-15)", "", "![](e_model_parallel.png)", "",
              "| variant | ranks | step ms | last loss | test accuracy |", "|---|---|---|---|---|"]
        for k, v in R["e"].items():
            acc = v["test_accuracy"]
            L.append(f"| {k} | {v['ranks']} | {v['step_ms']:.2f} | "
                     f"{(v['loss'] or [float('nan')])[-1]:.3f} | "
                     f"{'-' if acc is None else f'{acc:.3f}'} |")
        L += ["", "All four runs use the same seed, data order and optimiser (SGD lr 0.01, momentum "
              "0.9, batch 32). The two pipeline runs match each other (micro-batch gradients "
              "accumulate to the full-batch gradient); the RPC placement (reference programming "
              "model: driver + 2 stage owners over TensorPipe, `codes/task4/model.py`) and the "
              "tensor-parallel head reach the same loss and accuracy. The step times here include "
              "the process-group path of this device; the transport-level numbers for the "
              "pipeline (RCCL and xGMI transports, GPipe/1F1B, bubble fraction) are in "
              "`profiles/bench_pipeline_r3.jsonl` (`tools/bench_pipeline.py`).", ""]
    (out / "REPORT.md").write_text("\n".join(L))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", default=str(ROOT / "profiles" / "labs"))
    ap.add_argument("--device", default="cpu", choices=["cpu", "cuda"])
    ap.add_argument("--only", default="a,b,c,d,e")
    ap.add_argument("--world-sizes", default="2,4,8")
    ap.add_argument("--steps1", type=int, default=300)  # one epoch at batch 200
    ap.add_argument("--steps2", type=int, default=60)
    ap.add_argument("--steps3", type=int, default=40)
    ap.add_argument("--steps4", type=int, default=300)
    ap.add_argument("--steps5", type=int, default=300)
    a = ap.parse_args(argv)
    a.world_sizes = [int(w) for w in a.world_sizes.split(",")]
    global _SHARED_GPU
    if a.device == "cuda":
        import torch

        _SHARED_GPU = torch.cuda.device_count() < max(a.world_sizes + [3])
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    exps = {"a": exp_optimizers, "b": exp_comm, "c": exp_straggler, "d": exp_sampling,
            "e": exp_model_parallel}
    R = {}
    prev = out / "results.json"
    if prev.exists():
        R = json.loads(prev.read_text())
    for k in a.only.split(","):
        t0 = time.perf_counter()
        R[k] = exps[k](a, out)
        print(f"[lab_report] ({k}) done in {time.perf_counter() - t0:.1f} s", flush=True)
        prev.write_text(json.dumps(R, indent=1))
    write_report(out, R, a)
    print(f"[lab_report] wrote {out / 'REPORT.md'}")


if __name__ == "__main__":
    main()

"""Round-6 CPU tests: the lab-4 xGMI stage transport falls back to process-group P2P on
every rank together when peer-memory mapping fails on ONE rank (VERDICT r5 note A), and the
pipeline stage's replay() guard."""
import json
import time

import pytest


class _FakeLib:
    """Stand-in for the native library's IPC entry points: allocation and export succeed,
    opening a peer's handle fails on ``bad_rank`` only (the cross-GPU failure mode)."""

    def __init__(self, rank, bad_rank, fail="open"):
        self.rank, self.bad, self.fail = rank, bad_rank, fail
        self.n = 0
        self.closed, self.freed = [], []

    def xgmi_alloc(self, nbytes):
        if self.fail == "alloc" and self.rank == self.bad:
            raise RuntimeError("hipMalloc failed (injected)")
        self.n += 1
        return 4096 * self.n

    def xgmi_get_handle(self, base):
        return bytes(64)

    def xgmi_open_handle(self, h):
        if self.fail == "open" and self.rank == self.bad:
            raise RuntimeError("hipIpcOpenMemHandle: invalid argument (injected)")
        self.n += 1
        return 1 << 40 | self.n

    def xgmi_close_handle(self, p):
        self.closed.append(p)

    def xgmi_free(self, p):
        self.freed.append(p)


def _task4_xgmi_fallback(rank, ws, out_dir, fail):
    from dmlab.ops import _native
    from dmlab.tasks import task4

    fake = _FakeLib(rank, bad_rank=1, fail=fail)
    _native.lib = lambda: fake
    t0 = time.perf_counter()
    task4.main(["--mode", "pipeline", "--n_devices", str(ws), "--rank", str(rank),
                "--device", "cpu", "--synthetic", "--epochs", "1", "--max-steps", "3",
                "--no-test", "--transport", "xgmi", "--train-samples", "256",
                "--bench-json", f"{out_dir}/b.json"])
    dt = time.perf_counter() - t0
    assert dt < 60, f"fallback took {dt:.1f} s"
    # the rank that mapped its peer's buffers released them again
    if rank == 0 and fail == "open":
        assert fake.closed and len(fake.freed) == 2


@pytest.mark.parametrize("fail", ["open", "alloc"])
def test_task4_xgmi_mapping_failure_on_one_rank_falls_back_to_pg(tmp_path, fail):
    from dist_helpers import run_dist

    run_dist(_task4_xgmi_fallback, 2, str(tmp_path), fail)
    for r in range(2):
        res = json.loads((tmp_path / f"b.json.rank{r}").read_text())
        assert res["transport_used"] == "pg", res
        assert res["transport"] == "pg" and res["p2p_selfcheck"] == "pass"
        assert res["xgmi_p2p_selfcheck"] == "FAIL"
        assert "construction" in res["xgmi_p2p_reason"]
        assert "injected" in res["xgmi_p2p_reason"]


def _xgmi_allreduce_alloc_failure(rank, ws):
    import torch

    from dmlab.parallel import selfcheck, xgmi

    fake = _FakeLib(rank, bad_rank=ws - 1, fail="alloc")
    xgmi.lib = lambda: fake
    with pytest.raises(RuntimeError, match="injected"):
        xgmi.XGMIAllReduce(cap=1024, device=torch.device("cpu"))
    # the self-check built on it agrees on RCCL on every rank instead of hanging
    r = selfcheck.xgmi_selfcheck(torch.device("cpu"))
    assert r["small_allreduce_used"] == "rccl"


def test_xgmi_allreduce_alloc_failure_on_one_rank_raises_everywhere():
    from dist_helpers import run_dist

    run_dist(_xgmi_allreduce_alloc_failure, 2)


def _p2p_not_ready(rank, ws):
    import torch

    from dmlab.parallel import selfcheck

    class Half:
        """A transport whose channel to the peer exists on rank 0 only."""
        chan = {(0, 1): None, (1, 0): None} if rank == 0 else {}

        def send(self, *a):
            raise AssertionError("no message may be posted when a side is not ready")

        recv = send

    t0 = time.perf_counter()
    r = selfcheck.p2p_selfcheck(Half(), rank, 1 - rank, torch.device("cpu"), first=rank == 0)
    assert r == {"p2p_selfcheck": "FAIL"}
    assert time.perf_counter() - t0 < 30


def test_p2p_selfcheck_one_side_not_ready_fails_fast():
    from dist_helpers import run_dist

    run_dist(_p2p_not_ready, 2)


def test_pipeline_replay_before_capture_is_a_clear_error():
    from dmlab.parallel.pipeline import PipelineStage

    st = PipelineStage.__new__(PipelineStage)
    st._graph = None
    st.first = True
    with pytest.raises(RuntimeError, match="capture"):
        st.replay()

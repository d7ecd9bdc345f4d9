"""bench.py's report() aggregation on CPU (no kernels run): the SpMM roofline sums the algorithmic bytes
of every rank over the slowest rank's SpMM time, and the RCCL exchanges' HIP-event spans become the
`exchange_overlap` record (span, exposed wait, hidden fraction per rank)."""
import os
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]


def _kern(scale):
    # TIMER.summary() form: {(kind, M, N, F, tag): (launches, total ms)}
    return {("spmm", 100, 200, 64, "torch.float32"): (4, 2.0 * scale),
            ("fc", 100, 64, 64, "lin-x3"): (2, 1.0),
            ("exchange", 10, 12, 64, "span"): (5, 3.0 * scale),
            ("exchange", 10, 12, 64, "exposed"): (5, 0.6 * scale)}


def _report(rank, world, scale):
    import bench

    ctx = bench.Ctx(rank, world, "cpu", "gloo" if world > 1 else "none", world > 1)
    return bench.report(ctx, 1.0 * scale, _kern(scale), {}, steps=2, hids=64, local_nnz=1000, esz=4,
                        traffic_key="(none)")


def test_report_exchange_overlap_one_rank():
    out = _report(0, 1, 1.0)
    ex = out["exchange_overlap"]
    assert ex["per_rank"][0]["exchanges_per_step"] == 2.5
    assert abs(ex["per_rank"][0]["span_ms_per_step"] - 1.5) < 1e-12
    assert abs(ex["per_rank"][0]["exposed_ms_per_step"] - 0.3) < 1e-12
    assert abs(ex["per_rank"][0]["hidden_frac"] - 0.8) < 1e-12
    assert not any(k.startswith("exchange") for k in out["kernels"])  # not a kernel line
    assert out["roofline"]["launches"] == 4


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = _report(rank, world, 1.0 + rank)  # rank 1 twice as slow
        if rank == 0:
            ex = out["exchange_overlap"]
            assert len(ex["per_rank"]) == 2
            assert abs(ex["max_exposed_ms_per_step"] - 0.6) < 1e-12
            # value: both ranks' edges over the slowest rank's time (2 s)
            assert abs(out["value"] - 2 * 4 * 1000 / 2.0) < 1e-9
            # roofline: the sum of the bytes over (N x the slowest SpMM time)
            import bench

            b = 4 * bench.spmm_bytes(100, 1000, 64, 4)
            assert abs(out["roofline"]["achieved"] - 2 * b / (2 * 4.0 / 1e3) / 1e9) < 1e-6
            open(os.path.join(out_dir, "ok"), "w").write("ok")
    finally:
        dist.destroy_process_group()


def test_report_aggregates_over_ranks(tmp_path):
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    assert (tmp_path / "ok").exists()


if __name__ == "__main__":
    sys.exit(pytest.main([__file__, "-q"]))

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


# ---------------------------------------------------------------- the driver-parsed headline line
def _full_record(world=1, src="r05"):
    """A full bench record as main() builds it, widened to `world` ranks for the N > 1 shape: round 5's final
    default line (every sub-record with its kernel table, 20.9 KB), or ("r06") the detail file of a round-6
    default run (tests/data/bench_detail_r06.json: per-direction compulsory / counter-bytes fractions and
    their `bound` labels, which the first round-6 summary choked on)."""
    import copy
    import json

    if src == "r06":
        out = json.load(open(os.path.join(ROOT, "tests", "data", "bench_detail_r06.json")))
    else:
        path = os.path.join(ROOT, "profiles", "r05_bench_default_final.log")
        line = [ln for ln in open(path).read().splitlines() if ln.startswith("{")][-1]
        out = json.loads(line)
        out["arith"] = "f16x2"
    if world > 1:
        out = copy.deepcopy(out)
        out["n_gpus"] = world
        r0 = out["dist"]["ranks"][0]
        out["dist"]["ranks"] = [dict(r0, rank=r, local_rank=r, device=f"cuda:{r}", pci="0000:%02x:00" % (0x10 + r))
                                for r in range(world)]
        out["roofline"]["per_rank"] = [{"frac": 0.95, "avg_launch_ms": 1.1, "launches": 80, "bytes_per_launch": 8.8e9}
                                       for _ in range(world)]
        out["exchange_overlap"] = {"what": "x" * 200, "max_exposed_ms_per_step": 0.31,
                                   "per_rank": [{"exchanges_per_step": 12, "span_ms_per_step": 3.0,
                                                 "exposed_ms_per_step": 0.3, "hidden_frac": 0.9}] * world}
        out["exchange"] = {"per_rank": [{"k": "v" * 300}] * world}
        for s in ("inference", "inference_fp16", "c5", "skewed"):
            out.pop(s, None)
    return out


REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "arith", "data", "config", "dist", "roofline", "fc_roofline")


@pytest.mark.parametrize("world,src", [(1, "r05"), (8, "r05"), (1, "r06"), (8, "r06")])
def test_headline_is_compact_and_parses(world, src):
    """The line the driver parses: under 8 KB whole (the driver keeps the last ~8 KB of stdout+stderr and
    returned parsed:null for round 5's 20.9 KB line), valid JSON, the contract's keys, the roofline with
    its PMC traffic, the CPU baseline at N=1, one summary per sub-record, and no kernel tables."""
    import json

    import bench

    out = _full_record(world, src)
    assert len(json.dumps(out)) > 8192 or world > 1  # the full record alone would not fit
    line = json.dumps(bench.compact_headline(out, "gpurun_out/bench_detail.json"))
    assert len(line.encode()) < bench.HEADLINE_MAX_BYTES <= 8192, len(line)
    head = json.loads(line)
    for k in REQUIRED:
        assert k in head, k
    assert head["value"] == pytest.approx(out["value"], rel=1e-6)
    assert head["ms_per_step"] == pytest.approx(out["ms_per_step"], rel=1e-6)
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in head["roofline"], k
    assert head["roofline"]["frac"] == pytest.approx(out["roofline"]["frac"], rel=1e-5)
    assert "kernels" not in head and "kernels" not in json.dumps(head["subs"] if "subs" in head else {})
    assert len(head["dist"]["pci"]) == world
    if world == 1:
        cb = head["cpu_baseline"]
        for k in ("value", "unit", "cores", "kind", "sample"):
            assert k in cb, k
        assert set(head["subs"]) == {"c4", "inference", "inference_fp16", "c5", "skewed"}
        assert head["subs"]["c5"]["ms_per_step"] == pytest.approx(out["c5"]["ms_per_step"], rel=1e-4)
        assert "cpu_s" in head["subs"]["c5"]
        if src == "r06":  # the skewed directions' three fractions and their bound labels
            for dd in head["subs"]["skewed"]["dirs"].values():
                assert {"roofline_frac", "compulsory_frac", "traffic_frac", "bound"} <= set(dd), dd
                assert isinstance(dd["bound"], str)
    else:
        assert head["exchange_overlap"]["max_exposed_ms_per_step"] == pytest.approx(0.31)
        assert len(head["roofline"]["per_rank_frac"]) == world


def test_emit_prints_headline_last_and_writes_detail(tmp_path, capsys, monkeypatch):
    """emit(): the full record goes to the detail file (every sub-record and kernel table), the compact line
    is the LAST line of stdout and names the file."""
    import json

    import bench

    out = _full_record(1, "r06")
    detail = tmp_path / "d" / "bench_detail.json"
    monkeypatch.setenv("LPGNN_BENCH_DETAIL", str(detail))
    print("some earlier output")
    bench.emit(out, None)
    lines = capsys.readouterr().out.strip().splitlines()
    head = json.loads(lines[-1])
    assert head["detail"] == str(detail)
    full = json.load(open(detail))
    assert full["c5"]["kernels"] and full["skewed"]["kernels"]


def test_emit_survives_a_summary_failure(tmp_path, capsys, monkeypatch):
    """A bug in the compact summary still leaves a parseable last line with the contract's keys."""
    import json

    import bench

    out = _full_record(1, "r06")
    monkeypatch.setenv("LPGNN_BENCH_DETAIL", str(tmp_path / "bench_detail.json"))
    monkeypatch.setattr(bench, "compact_headline", lambda *a: 1 / 0)
    bench.emit(out, None)
    head = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert head["value"] == out["value"] and head["roofline"]["frac"] == out["roofline"]["frac"]

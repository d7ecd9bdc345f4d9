"""The run_exp / validation driver (lpgnn.run, train.py:55-157, val.py:43-68)
with the real GCN_FC on the HIP path: a 2-epoch run on synthetic .pk LPs
(one of them above the edge threshold, so it trains through the k-hop
NeighborLoader), checkpoint compatibility with the reference's key set,
the per-epoch LR schedule, validation, and the 16-bit (--fp16) route."""
import os

import numpy as np
import pytest
import torch

from oracle import model_ref as O
from tests.test_run import write_dataset

pytestmark = pytest.mark.gpu


def _args(tmp_path, *extra):
    from lpgnn import run

    a = run.parse_args(["train", "--arch", "GCN_FC(8,8,hids=64,depth=3)", "--dataset", "synth", "--data_prefix",
                        str(tmp_path / "data"), "--log_prefix", str(tmp_path / "runs"), "--epochs", "2",
                        "--edge_num_thresh", "700", "--batch_size", "64", *extra])
    return a


def test_run_exp_two_epochs_checkpoint_and_validation(tmp_path):
    from lpgnn import GCN_FC, batch_to, run

    # graphs of 600, 500, 800 (> threshold 700: NeighborLoader path) and 400 edges
    write_dataset(str(tmp_path / "data" / "synth" / "highs-inp_tgt"), k=4)
    args = _args(tmp_path)
    ds = run.LPDataset(args.dataset_processed_prefix, thresh_num=args.edge_num_thresh, device=args.dev)
    tr, va = run.split_train_val(ds)
    assert [os.path.basename(tr.path(i)) for i in range(len(tr))] == ["lp2.pk", "lp3.pk"]  # seed-0 70/30 split
    hist = run.run_exp(args)
    assert hist["lr"] == [1e-3, 1e-4]
    assert all(np.isfinite(hist["epoch_loss"]))
    # lp2 (800 edges) went through the sampler in mini-batches of 64 seeds: more steps than graphs
    assert hist["steps"] > 2 * 2
    ck = torch.load(hist["checkpoint"], map_location="cpu", weights_only=True)
    ref = O.init_state_dict(8, 8, 64, 3)
    assert list(ck.keys()) == list(ref.keys()) and all(ck[k].shape == ref[k].shape for k in ref)
    # --load_from + validation (full graph and k-hop every-neighbour inference)
    vargs = _args(tmp_path, "--load_from", hist["checkpoint"])
    model = run.make_model(vargs)
    for k, v in ck.items():
        assert torch.equal(model.state_dict()[k].cpu(), v)
    _, acc, rows = run.validation(model, ds, vargs)
    assert 0.0 <= acc <= 1.0 and len(rows) == 4
    # --fp16: model.half() on the evaluation model (val.py:269), every batch through batch_to(half=True);
    # training stays fp32 whatever the flag (the reference's train.py never reads it); logits close to
    # the fp32 model's
    fargs = _args(tmp_path, "--load_from", hist["checkpoint"], "--fp16", "1")
    assert next(run.make_model(fargs).parameters()).dtype == torch.float32
    m16 = run.make_model(fargs, for_eval=True)
    assert next(m16.parameters()).dtype == torch.float16
    _, acc16, _ = run.validation(m16, ds, fargs)
    assert 0.0 <= acc16 <= 1.0
    g = ds[0].to(args.dev)
    with torch.no_grad():
        a = torch.cat(model.eval()(g))
        b = torch.cat(m16.eval()(batch_to(g, args.dev, half=True)))
    assert b.dtype == torch.float16 and (a - b.float()).abs().mean().item() < 0.05


def test_half_model_trains_refused_eval_runs():
    """val.py:269 model.half() / batch_to(half=True) is the reference's inference mode: eval runs on the
    fp16 kernels (fp16 logits); a training forward is refused with a clear error (the reference never
    trains in fp16)."""
    from lpgnn import BipartiteBatch, BipartiteCSR, GCN_FC, batch_to, synth

    g = synth.uniform_lp(50, 80, 400, seed=1)
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device="cuda:0")
    b = BipartiteBatch(x_s=torch.from_numpy(g.x_s), x_t=torch.from_numpy(g.x_t), y_s=torch.from_numpy(g.y_s),
                       y_t=torch.from_numpy(g.y_t), edge_index=adj, s_bs=g.m, t_bs=g.n)
    model = GCN_FC(8, 8, hids=32, depth=3).cuda().half().eval()
    with torch.no_grad():
        lc, lv = model(batch_to(b, "cuda:0", half=True))
    assert lc.dtype == torch.float16 and torch.isfinite(lc).all() and torch.isfinite(lv).all()
    with pytest.raises(RuntimeError, match="inference mode"):
        model.train()(b)


def _partition_worker(rank, world, port, tmp, epochs):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)  # ranks share the box's one GPU
    try:
        from lpgnn import GCN_FC, run

        args = run.parse_args(["train", "--arch", "GCN_FC(8,8,hids=64,depth=3)", "--dataset", "synth",
                               "--data_prefix", os.path.join(tmp, "data"), "--log_prefix", os.path.join(tmp, "runs"),
                               "--epochs", str(epochs), "--edge_num_thresh", "700", "--partition", "1"])
        torch.manual_seed(0)
        model = GCN_FC(8, 8, hids=64, depth=3).to(args.dev)  # dp 0.1: masks keyed on global node ids
        torch.manual_seed(1)
        hist = run.run_exp(args, model=model)
        ds = run.LPDataset(args.dataset_processed_prefix, thresh_num=args.edge_num_thresh, device=args.dev)
        _, acc, _ = run.validation(model, ds, args)
        # --fp16 evaluation of the same graphs (val.py:269 model.half()): the partitioned ones on the fp16
        # partitioned layers (lpgnn.partition._part_forward_f16)
        import copy

        _, acc16, _ = run.validation(copy.deepcopy(model).half(), ds, args)
        torch.save({"loss": hist["epoch_loss"], "acc": float(acc), "acc16": float(acc16),
                    "sd": {k: v.cpu() for k, v in model.state_dict().items()}}, os.path.join(tmp, f"part{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_run_partition_two_hip_ranks_match_one_gpu(tmp_path):
    """``run.py train --partition 1`` with 2 HIP ranks (gloo, sharing the GPU) on .pk LPs above
    --edge_num_thresh (800 and 1800 edges vs 700): every epoch's loss and the final parameters equal the
    one-GPU full-graph training of the same model and seeds (dropout 0.1 -- the masks are keyed on
    global node ids) within fp32 summation-order tolerance; both ranks end bitwise identical;
    validation over every graph (partitioned above the threshold) gives the one-GPU accuracy."""
    import socket

    import torch.multiprocessing as mp

    from lpgnn import GCN_FC, run

    write_dataset(str(tmp_path / "data" / "synth" / "highs-inp_tgt"), k=4,
                  sizes=((60, 120, 600), (50, 90, 500), (80, 100, 800), (90, 200, 1800)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_partition_worker, args=(2, port, str(tmp_path), 3), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "part0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "part1.pt", weights_only=True)
    for k in r0["sd"]:
        assert torch.equal(r0["sd"][k], r1["sd"][k]), k
    # one GPU, whole graphs (no threshold: every graph one full-graph step)
    args = run.parse_args(["train", "--arch", "GCN_FC(8,8,hids=64,depth=3)", "--dataset", "synth", "--data_prefix",
                           str(tmp_path / "data"), "--log_prefix", str(tmp_path / "runs1"), "--epochs", "3",
                           "--edge_num_thresh", "1e12"])
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=64, depth=3).to(args.dev)
    torch.manual_seed(1)
    hist = run.run_exp(args, model=model)
    print("partitioned epoch losses", r0["loss"], "one GPU", hist["epoch_loss"])
    np.testing.assert_allclose(r0["loss"], hist["epoch_loss"], rtol=1e-5)
    worst = 0.0
    for k, v in model.state_dict().items():
        d = (r0["sd"][k] - v.cpu()).abs().max().item()
        worst = max(worst, d)
        np.testing.assert_allclose(r0["sd"][k].numpy(), v.cpu().numpy(), rtol=1e-4, atol=2e-6, err_msg=k)
    ds = run.LPDataset(args.dataset_processed_prefix, device=args.dev)
    _, acc, _ = run.validation(model, ds, args)
    print(f"max |param_partitioned - param_one_gpu| {worst:.2e}; accuracy {r0['acc']:.6f} vs {acc:.6f}")
    assert abs(r0["acc"] - acc) < 1e-9 and abs(r1["acc"] - acc) < 1e-9
    # --fp16 validation: the partitioned graphs' fp16 logits differ from one GPU's only where a boundary
    # variable's reordered fp32 sum rounds to another fp16 value -- the accuracy agrees to a label or two
    import copy

    _, acc16, _ = run.validation(copy.deepcopy(model).half(), ds, args)
    print(f"fp16 accuracy partitioned {r0['acc16']:.6f} / {r1['acc16']:.6f} vs one GPU {acc16:.6f}")
    assert r0["acc16"] == r1["acc16"] and abs(r0["acc16"] - acc16) <= 0.01

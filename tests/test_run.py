"""The run_exp / validation driver and CLI (lpgnn.run) on the host: dataset
layout and split, LR schedule, checkpoints, and the data-parallel replicas
over gloo.  The product model needs the GPU, so these tests drive the loop
with a small stand-in module of the same API (forward(batch) -> logits);
tests/test_gpu_run.py runs the same driver with GCN_FC on the device."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def write_dataset(root, k=4, seed=0, sizes=((60, 120, 600), (50, 90, 500), (80, 100, 800), (40, 70, 400))):
    """k synthetic LPs as processed .pk records (dataset.py:213-217 layout)
    under {root}/processed, named like the reference's files."""
    from lpgnn import lpio, synth

    os.makedirs(os.path.join(root, "processed"), exist_ok=True)
    for i in range(k):
        m, n, nnz = sizes[i % len(sizes)]
        g = synth.uniform_lp(m, n, nnz, seed=seed + i)
        rec = [g.row.astype(np.int32), g.col.astype(np.int32), g.val.astype(np.float64), g.x_s, g.x_t, g.y_s, g.y_t,
               m + n]
        lpio.msgpack_dump(rec, os.path.join(root, "processed", f"lp{i}.pk"))
    return root


class TinyModel(torch.nn.Module):
    """Stand-in with GCN_FC's call contract (and GCNBase save/load)."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.lin_left = torch.nn.Linear(8, 3)
        self.lin_right = torch.nn.Linear(8, 3)

    def forward(self, batch):
        return self.lin_left(batch.x_s), self.lin_right(batch.x_t)

    def save(self, pn):
        torch.save(self.state_dict(), pn)

    def load(self, pn):
        self.load_state_dict(torch.load(pn, map_location="cpu", weights_only=True))


def _args(tmp_path, *extra):
    from lpgnn import run

    return run.parse_args(["train", "--dataset", "synth", "--data_prefix", str(tmp_path / "data"), "--log_prefix",
                           str(tmp_path / "runs"), "--epochs", "2", "--exp_nm", "t", *extra])


def test_cli_flags_and_paths(tmp_path):
    from lpgnn import run

    a = run.parse_args(["val", "--arch", "GCN_FC(8,8,hids=1024,depth=3)", "--dataset", "mirp", "--data_prefix", "/d",
                        "--lp_method", "primal", "--solver_prefix", "highs", "--fp16", "1"])
    assert a.phase == "val" and a.lp_method == 4 and a.fp16 == 1
    assert a.dataset_processed_prefix == "/d/mirp/highs-inp_tgt-m4/"  # utils.py:836-837
    assert a.edge_num_thresh == 12e6 and a.batch_size == 327680  # utils.py:812-813
    b = run.parse_args([])
    assert b.phase == "train" and b.lr == 1e-3 and b.opt == "adam" and b.loss == "balanced"
    assert b.dataset_processed_prefix.endswith("/None/highs-inp_tgt/")


def test_split_matches_reference_rule():
    """utils.py:256-262: int(max(0.7 n, 1)) train graphs from a seed-0 permutation."""
    from lpgnn import run

    for n in (1, 2, 3, 4, 10, 37):
        tr, va = run.split_idxs_train_val(n, 0)
        np.random.seed(0)
        p = np.random.permutation(n)
        k = int(max(n * 7 / 10, 1))
        assert np.array_equal(tr, np.sort(p[:k])) and np.array_equal(va, np.sort(p[k:]))


def test_dataset_order_and_loading(tmp_path):
    from lpgnn import run

    root = write_dataset(str(tmp_path / "ds"), k=4)
    for nm in ("lp10.pk", "lp2b.pk"):  # (len, name) ordering, dataset.py:164
        os.link(os.path.join(root, "processed", "lp1.pk"), os.path.join(root, "processed", nm))
    ds = run.LPDataset(root, device="cpu")
    assert [os.path.basename(ds.path(i)) for i in range(len(ds))] == \
        ["lp0.pk", "lp1.pk", "lp2.pk", "lp3.pk", "lp10.pk", "lp2b.pk"]
    b = ds[1]
    assert hasattr(b, "x_s") and b.x_s.shape == (50, 8) and b.edge_index.nnz() == 500
    small = run.LPDataset(root, device="cpu", thresh_num=450)  # above the threshold: homogeneous graph
    assert not hasattr(small[1], "x_s") and small[1].num_nodes == 140 and hasattr(small[3], "x_s")
    sub = ds[np.array([3, 0])]
    assert len(sub) == 2 and os.path.basename(sub.path(0)) == "lp3.pk"


def test_run_exp_schedule_checkpoint_and_resume(tmp_path):
    from lpgnn import run

    write_dataset(str(tmp_path / "data" / "synth" / "highs-inp_tgt"), k=4)
    args = _args(tmp_path)
    args.dev = "cpu"
    hist = run.run_exp(args, model=TinyModel())
    assert hist["lr"] == [1e-3, 1e-4]  # StepLR(step_size=max(2 // 4, 1), gamma=0.1), stepped per epoch
    assert hist["steps"] == 2 * 2 and all(np.isfinite(hist["epoch_loss"]))  # 2 train graphs x 2 epochs
    ck = torch.load(hist["checkpoint"], map_location="cpu", weights_only=True)
    assert set(ck) == set(TinyModel().state_dict())
    assert os.path.exists(os.path.join(args.log_dir, "args.json"))
    # --load_from resumes from the checkpoint
    m2 = TinyModel()
    m2.load(hist["checkpoint"])
    for k, v in ck.items():
        assert torch.equal(m2.state_dict()[k], v)
    # validation on the held-out graphs
    ds = run.LPDataset(args.dataset_processed_prefix, device="cpu")
    _, va = run.split_train_val(ds)
    import lpgnn.val as V

    real = V.model_inference_with_batch
    try:
        V.model_inference_with_batch = lambda model, g, *a, **k: model(g)
        _, acc, rows = run.validation(m2, va, args)
    finally:
        V.model_inference_with_batch = real
    assert 0.0 <= acc <= 1.0 and len(rows) == 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _replica_worker(rank, world, port, tmp):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    try:
        from lpgnn import run

        args = run.parse_args(["train", "--dataset", "synth", "--data_prefix", os.path.join(tmp, "data"),
                               "--log_prefix", os.path.join(tmp, f"runs{rank}"), "--epochs", "1", "--replicas", "1"])
        args.dev = "cpu"
        model = TinyModel()
        run.run_exp(args, model=model)
        torch.save(model.state_dict(), os.path.join(tmp, f"final{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_data_parallel_replicas_gloo(tmp_path):
    """2 gloo ranks, 4 graphs -> 2 train graphs = one round: both ranks end
    with identical parameters, equal to one Adam step on the mean of the two
    graphs' gradients (computed here in one process)."""
    from lpgnn import run
    from lpgnn.train import balanced, make_optimizer

    write_dataset(str(tmp_path / "data" / "synth" / "highs-inp_tgt"), k=4)
    mp.spawn(_replica_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    p0 = torch.load(tmp_path / "final0.pt", weights_only=True)
    p1 = torch.load(tmp_path / "final1.pt", weights_only=True)
    for k in p0:
        assert torch.equal(p0[k], p1[k]), k
    # reference: same init, mean gradient of the two train graphs, one Adam step
    args = _args(tmp_path)
    ds = run.LPDataset(args.dataset_processed_prefix, device="cpu")
    tr, _ = run.split_train_val(ds)
    model = TinyModel()
    opt, _ = make_optimizer(model, "adam", 1e-3, 1)
    grads = []
    for i in range(len(tr)):
        model.zero_grad()
        b = tr[i]
        lc, lv = model(b)
        balanced(lc, lv, b.y_s, b.y_t).backward()
        grads.append([p.grad.clone() for p in model.parameters()])
    for p, ga, gb in zip(model.parameters(), *grads):
        p.grad = (ga + gb) / 2
    opt.step()
    for k, v in model.state_dict().items():
        torch.testing.assert_close(p0[k], v, rtol=1e-6, atol=1e-7, msg=k)


def test_fp16_flag_is_validation_only(tmp_path):
    """--fp16 (utils.py:770) changes only the evaluation model (val.py:269 model.half()):
    train.py trains in fp32 whatever the flag, and so does run_exp's model."""
    from lpgnn import run

    dt = lambda m: next(m.parameters()).dtype  # noqa: E731
    a = _args(tmp_path, "--fp16", "1", "--arch", "GCN_FC(8,8,hids=16,depth=3)")
    assert dt(run.make_model(a)) == torch.float32
    assert dt(run.make_model(a, for_eval=True)) == torch.float16
    b = _args(tmp_path, "--arch", "GCN_FC(8,8,hids=16,depth=3)")
    assert dt(run.make_model(b, for_eval=True)) == torch.float32


def test_dataset_reads_each_graph_once(tmp_path, monkeypatch):
    """LPDataset decodes a .pk file once per __getitem__ (the nnz threshold test reuses the record)."""
    from lpgnn import lpio, run

    root = write_dataset(str(tmp_path / "data"))
    ds = run.LPDataset(root)
    calls = []
    real = lpio.msgpack_load
    monkeypatch.setattr(lpio, "msgpack_load", lambda p: calls.append(p) or real(p))
    g = ds[1]
    assert len(calls) == 1 and hasattr(g, "x_s")
    assert ds.nnz(1) == g.edge_index.nnz() and len(calls) == 1


def test_world_size_without_replicas_is_refused(tmp_path, monkeypatch):
    """Under a launcher (WORLD_SIZE > 1) without --replicas every rank would train the whole
    schedule into the same log directory: main() refuses."""
    from lpgnn import run

    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="--replicas"):
        run.main(["train", "--dataset", "synth", "--data_prefix", str(tmp_path / "d"), "--log_prefix",
                  str(tmp_path / "r")])


# ---------------------------------------- --partition: large graphs row-partitioned over the ranks
def _oracle_swaps():
    """The product's HIP local compute -> the oracle (tests/test_partition.py's doubles)."""
    import torch.nn.functional as F

    import lpgnn.fc as fc
    import lpgnn.partition as part
    from oracle import model_ref as O

    def spmm(adj, x):
        fwd = (adj.fwd.rowptr.numpy(), adj.fwd.col.numpy(), adj.fwd.val.numpy())
        bwd = (adj.bwd.rowptr.numpy(), adj.bwd.col.numpy(), adj.bwd.val.numpy())
        return O.spmm_t(fwd, bwd, x)

    def conv_fc(agg, x_dst, w_rel, b_rel, w_root, relu, dropout=0.0, row_offset=0, row_keys=None, arith=None):
        out = F.linear(agg, w_rel, b_rel) + F.linear(x_dst, w_root)
        return torch.relu(out) if relu else out

    def knowledge(logit, feas, bound=10):
        return O.add_knowledge(logit, logit[:1], feas, feas[:1], bound)[0]

    part._local_spmm = spmm
    fc.graph_conv_fc = conv_fc
    fc.linear = lambda x, w, b, fold_in=False, opts=None: F.linear(x, w, b)
    fc.knowledge = knowledge


PART_SIZES = ((120, 260, 1800), (90, 200, 1350))


def _partition_worker(rank, world, port, tmp, thresh):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    try:
        from lpgnn import GCN_FC, run

        _oracle_swaps()
        args = run.parse_args(["train", "--dataset", "synth", "--data_prefix", os.path.join(tmp, "data"),
                               "--log_prefix", os.path.join(tmp, "runs"), "--epochs", "3", "--partition", "1",
                               "--edge_num_thresh", str(thresh), "--arch", "GCN_FC(8,8,hids=16,depth=3)"])
        args.dev = "cpu"
        torch.manual_seed(0)
        model = GCN_FC(8, 8, hids=16, depth=3, dp=0.0)
        hist = run.run_exp(args, model=model)
        ds = run.LPDataset(args.dataset_processed_prefix, thresh_num=args.edge_num_thresh, device="cpu")
        _, va = run.split_train_val(ds)
        _, acc, rows = run.validation(model, va, args)
        torch.save({"loss": hist["epoch_loss"], "acc": float(acc), "sd": model.state_dict()},
                   os.path.join(tmp, f"part{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_run_partition_gloo_matches_one_process(tmp_path):
    """``run.py train --partition 1`` under 2 gloo ranks on a dataset whose graphs are above
    --edge_num_thresh (oracle local compute): every epoch's loss and the final parameters equal a
    one-process full-graph training of the same model (the oracle's forward, balanced loss, Adam +
    StepLR, train.py:85-157) within fp32 summation-order tolerance, both ranks end bitwise
    identical, rank 0's mdl.pth is that model, and ``validation`` (gathered logits, the reference's
    accuracy) gives the one-process accuracy."""
    from lpgnn import GCN_FC, run
    from lpgnn.val import accuracy
    from oracle import model_ref as O

    write_dataset(str(tmp_path / "data" / "synth" / "highs-inp_tgt"), k=2, sizes=PART_SIZES)
    mp.spawn(_partition_worker, args=(2, _free_port(), str(tmp_path), 1000), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "part0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "part1.pt", weights_only=True)
    for k in r0["sd"]:
        assert torch.equal(r0["sd"][k], r1["sd"][k]), k
    ck = torch.load(tmp_path / "runs" / "tmp" / "mdl.pth", weights_only=True)
    for k in ck:
        assert torch.equal(ck[k], r0["sd"][k]), k

    # one process, whole graph: the oracle's GCN_FC (MKL fp32), the same optimizer and schedule
    args = _args(tmp_path, "--epochs", "3")
    ds = run.LPDataset(args.dataset_processed_prefix, device="cpu")
    tr, va = run.split_train_val(ds)
    torch.manual_seed(0)
    params = {k: v.detach().clone().requires_grad_(True)
              for k, v in GCN_FC(8, 8, hids=16, depth=3, dp=0.0).state_dict().items()}
    opt = torch.optim.Adam(list(params.values()), lr=1e-3, weight_decay=5e-4)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=max(3 // 4, 1), gamma=0.1)

    def fwd(rec):
        row, col, val, xs, xt, ys, yt, _ = rec
        m, n = len(xs), len(xt)
        A = O.csr_from_coo(np.asarray(row), np.asarray(col), np.asarray(val, np.float32), m, n)
        AT = O.csr_transpose(*A, m, n)
        lc, lv = O.gcn_fc_forward(params, torch.as_tensor(np.asarray(xs)), torch.as_tensor(np.asarray(xt)), A, AT, 3)
        return lc, lv, torch.as_tensor(np.asarray(ys)), torch.as_tensor(np.asarray(yt))

    losses = []
    for _ in range(3):
        lc, lv, ys, yt = fwd(tr.record(0))  # one train graph (70 / 30 of 2)
        loss = O.balanced(lc, lv, ys, yt)
        opt.zero_grad()
        loss.backward()
        opt.step()
        sched.step()
        losses.append(loss.item())
    print("partitioned epoch losses", r0["loss"], "one process", losses)
    np.testing.assert_allclose(r0["loss"], losses, rtol=1e-5)
    for k, v in params.items():
        np.testing.assert_allclose(r0["sd"][k].numpy(), v.detach().numpy(), rtol=1e-4, atol=2e-6, err_msg=k)
    with torch.no_grad():
        lc, lv, ys, yt = fwd(va.record(0))
    acc = accuracy(torch.cat((lc, lv)), torch.cat((ys, yt)), lc.shape[0])
    assert abs(r0["acc"] - acc) < 1e-9 and abs(r1["acc"] - acc) < 1e-9, (r0["acc"], r1["acc"], acc)


def test_partition_flag_rules(tmp_path, monkeypatch):
    from lpgnn import run

    write_dataset(str(tmp_path / "data" / "synth" / "highs-inp_tgt"), k=2, sizes=PART_SIZES)
    a = _args(tmp_path, "--partition", "1", "--edge_num_thresh", "1500")
    ds = run.LPDataset(a.dataset_processed_prefix, device="cpu")
    assert [run._partitioned(a, ds, i) for i in range(2)] == [True, False]  # 1800 > 1500 >= 1350
    a.partition = 2
    assert all(run._partitioned(a, ds, i) for i in range(2))
    a.partition = 0
    assert not any(run._partitioned(a, ds, i) for i in range(2))
    b = _args(tmp_path, "--partition", "1", "--replicas", "1")
    b.dev = "cpu"
    monkeypatch.setattr(run, "_dist_world", lambda: (0, 2))  # replicas only engage at world > 1
    with pytest.raises(ValueError, match="exclusive"):
        run.run_exp(b, model=TinyModel())

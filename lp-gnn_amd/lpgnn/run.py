"""Training / evaluation driver and CLI: the reference's ``run_exp``
(train.py:55-157), ``validation`` (val.py:43-68) and flag set
(utils.py:743-770), on the HIP path.

    python -m lpgnn.run train --arch "GCN_FC(8,8,hids=1024,depth=3)" --dataset mirp --epochs 800
    python -m lpgnn.run val   --arch "GCN_FC(8,8,hids=1024,depth=3)" --dataset mirp --load_from runs/x/mdl.pth

What it keeps from the reference, flag for flag: the dataset directory
layout (``{data_prefix}/{dataset}/{solver_prefix}inp_tgt{-m<lp_method>}/``,
utils.py:836-837, holding the processed ``.pk`` files), the file order
(sorted by (len(name), name), dataset.py:160-168), the 70/30 seed-0
train/val split (utils.py:256-272), ``eval(args.arch)`` (safe:
arch.build_model), ``--load_from``, Adam/SGD with weight decay 5e-4 and
StepLR(epochs // 4, 0.1) stepped once per epoch, one graph per step
(DataLoader batch_size=1, shuffle=True), graphs above ``--edge_num_thresh``
cut into k-hop NeighborLoader mini-batches (fanout 6 for training, every
neighbour for evaluation), the NaN assert, the running loss/accuracy meters
(last-10 means, utils.py:874-899), ``mdl.pth`` written after every epoch
and ``args.json`` in the log directory.

What is different, and why:

* accuracy per step is computed on the device (val.accuracy_device, no host
  sync); the host sklearn path is used only by ``validation``;
* ``--fp16 1`` (utils.py:770; val.py:269 ``model.half()``) converts the
  VALIDATION model to fp16, as in the reference (train.py never converts the
  model), and every evaluated batch goes through ``batch_to(half=True)``
  (val.py:31): the fp16 kernels (fp16 storage, fp32 accumulation).  Training
  stays fp32 with the flag set;
* ``--replicas`` (torch.distributed initialised, world > 1): data parallel
  over graphs ("many small LPs: replicas only").  Every rank
  walks the same shuffled epoch order and takes every world-th graph; the
  parameter gradients are averaged with one bucketed all-reduce per round
  (a round = one graph per rank, all of that graph's mini-batches
  accumulated), so one optimizer step sees `world` graphs where the
  reference's sees one -- a larger effective batch, reported as such;
* ``--partition 1`` (torch.distributed initialised, or one process): the
  graphs above ``--edge_num_thresh`` -- which the reference cuts into
  NeighborLoader mini-batches on one device (train.py:103-116, val.py:19-27,
  utils.py:808) -- are trained and evaluated WHOLE, row-partitioned over the
  ranks (lpgnn.partition): every rank reads the .pk on the
  host, plans only its own constraint rows (partition.plan_partition_local),
  and one optimizer step per graph sees the full-graph gradient (the
  per-rank balanced-loss shares and parameter gradients are all-reduced), so
  the result is the one-GPU full-graph step's up to fp32 summation order.
  Graphs at or below the threshold run whole on every rank (identical
  replicated steps, no communication).  ``--partition 2``: every graph is
  row-partitioned.  Training uses the balanced loss (the published one); the
  logged accuracy and ``validation`` gather the owned rows' logits
  (partition.gather_logits) and apply the reference's rules to the whole graph.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys

import numpy as np
import torch

log = logging.getLogger("lpgnn.run")


# ------------------------------------------------------------------ dataset
class LPDataset:
    """LPDataset (dataset.py:99-264) over a directory of processed .pk files.

    ``root`` is the dataset_processed_prefix; files are looked up in
    ``root/processed`` (PyG's processed_dir), ``root/raw`` records are
    processed on first use (LPDataset.process, dataset.py:178-224).
    Indexing with an int returns the graph (a BipartiteBatch when
    nnz <= thresh_num, else the homogeneous graph for the NeighborLoader --
    MyToBipartite, dataset.py:280-281); with an index array, a subset."""

    def __init__(self, root, thresh_num=np.inf, device="cpu", indices=None, direct=True):
        self.root, self.thresh_num, self.device, self.direct = str(root), thresh_num, device, direct
        self.processed_dir = os.path.join(self.root, "processed")
        self.raw_dir = os.path.join(self.root, "raw")
        self._files = self._file_names()
        self._indices = list(range(len(self._files))) if indices is None else list(indices)
        self._nnz = {}  # file index -> edge count, learned on first load (shared by subsets)

    def _file_names(self):
        """dataset.py:160-168: the longer listing of raw/ and processed/,
        .pk files sorted by (len(name), name)."""
        fns = []
        for folder in (self.raw_dir, self.processed_dir):
            if not os.path.isdir(folder):
                continue
            now = sorted((f for f in os.listdir(folder) if f.endswith(".pk")), key=lambda nm: (len(nm), nm))
            if len(now) > len(fns):
                fns = now
        if not fns:
            raise ValueError(f"not found pk under {self.root}")
        self._process_missing(fns)
        return fns

    def _process_missing(self, fns):
        from . import lpio

        for fn in fns:
            dst = os.path.join(self.processed_dir, fn)
            if os.path.exists(dst):
                continue
            os.makedirs(self.processed_dir, exist_ok=True)
            lpio.msgpack_dump(lpio.process_raw(lpio.msgpack_load(os.path.join(self.raw_dir, fn))), dst)

    def __len__(self):
        return len(self._indices)

    def indices(self):
        return list(self._indices)

    def path(self, i: int) -> str:
        return os.path.join(self.processed_dir, self._files[self._indices[i]])

    def nnz(self, i: int) -> int:
        """Edge count of graph i (the file is read once; the count is cached)."""
        from . import lpio

        f = self._indices[i]
        if f not in self._nnz:
            self._nnz[f] = int(np.asarray(lpio.msgpack_load(self.path(i))[0]).shape[0])
        return self._nnz[f]

    def record(self, i: int):
        """Graph i's processed record [row, col, A_data, c_feas, v_feas, y_s, y_t, nnodes] (host arrays:
        the row-partitioned path plans and slices it per rank)."""
        from . import lpio

        rec = lpio.msgpack_load(self.path(i))
        self._nnz[self._indices[i]] = int(np.asarray(rec[0]).shape[0])
        return rec

    def __getitem__(self, idx):
        if isinstance(idx, (list, tuple, np.ndarray)):
            return LPDataset._subset(self, [self._indices[int(i)] for i in idx])
        from . import lpio

        i = int(idx)
        p = self.path(i)
        rec = lpio.msgpack_load(p)  # one read and decode per graph and epoch
        self._nnz[self._indices[i]] = int(np.asarray(rec[0]).shape[0])
        # above the threshold the reference keeps the homogeneous graph (dataset.py:280-281);
        # the direct loader packs the dual CSR on the device without the undirected round trip
        if self.direct and self._nnz[self._indices[i]] <= self.thresh_num:
            return lpio.load_bipartite(p, device=self.device, record=rec)
        return lpio.load_processed(p, device=self.device, thresh_num=self.thresh_num, record=rec)

    @staticmethod
    def _subset(ds, indices):
        sub = LPDataset.__new__(LPDataset)
        sub.__dict__.update(ds.__dict__)
        sub._indices = list(indices)
        return sub


def split_idxs_train_val(ngraphs: int, seed: int = 0):
    """utils.py:256-262."""
    ntrain = int(max(ngraphs * 7 / 10, 1))
    np.random.seed(seed)
    idxs = np.random.permutation(ngraphs)
    return np.sort(idxs[:ntrain]), np.sort(idxs[ntrain:])


def split_train_val(ds, seed: int = 0):
    """utils.py:265-272 (the seed is forced to 0, as there)."""
    if seed != 0:
        log.warning("seed for train val not 0, will force set to 0")
        seed = 0
    tr, va = split_idxs_train_val(len(ds), seed)
    log.info(f"split into {len(tr)} train {len(va)} val, seed: {seed}")
    return ds[tr], ds[va]


class AverageMeter:
    """utils.py:874-899 ("way 1": mean of the last 10 values)."""

    def __init__(self):
        import collections

        self.mem = collections.deque(maxlen=10)
        self.avg = 0.

    def reset(self):
        self.avg = 0.

    def update(self, val):
        self.mem.append(float(val))
        self.avg = float(np.mean(list(self.mem)))


# ------------------------------------------------------------------- flags
def parser():
    """utils.py:743-770 (+ preprecess_args defaults, utils.py:810-823)."""
    ap = argparse.ArgumentParser(prog="python -m lpgnn.run")
    ap.add_argument("phase", nargs="?", choices=("train", "val"), default="train")
    ap.add_argument("--dev", type=int, default=0)
    ap.add_argument("--exp_nm", type=str, default="tmp")
    ap.add_argument("--opt", type=str, default="adam")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--epochs", type=int, default=30)
    ap.add_argument("--arch", type=str, default="GCN_FC(8,8,hids=128)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--num_workers", type=int, default=0)
    ap.add_argument("--batch_size", type=int, default=10240 * 8 * 4)
    ap.add_argument("--load_from", type=str, default="None")
    ap.add_argument("--dataset", type=str, default="None")
    ap.add_argument("--solver_prefix", type=str, default="highs-")
    ap.add_argument("--data_prefix", type=str, default=os.path.abspath("./lp-dataset/"))
    ap.add_argument("--exist_ok", type=int, default=1)
    ap.add_argument("--edge_num_thresh", type=float, default=4e6 * 3)
    ap.add_argument("--verbose", type=int, default=1)
    ap.add_argument("--loss", type=str, default="balanced")
    ap.add_argument("--lp_method", type=str, default="1")
    ap.add_argument("--split", type=str, default="val")
    ap.add_argument("--log_prefix", type=str, default=os.path.abspath("./runs/"))
    ap.add_argument("--fp16", type=int, default=0)
    ap.add_argument("--prefetch_factor", type=int, default=2)
    ap.add_argument("--replicas", type=int, default=0,
                    help="data parallel over graphs when torch.distributed is initialised (world > 1)")
    ap.add_argument("--partition", type=int, default=0, choices=(0, 1, 2),
                    help="1: graphs above --edge_num_thresh are trained / evaluated whole, row-partitioned over "
                         "the ranks (instead of NeighborLoader mini-batches); 2: every graph is")
    return ap


def postprocess_args(args):
    """utils.py:825-842: dataset / processed / log paths, lp_method suffix."""
    if not args.solver_prefix.endswith("-"):
        args.solver_prefix += "-"
    lp_method = {"dual": 1, "primal": 4}.get(args.lp_method, args.lp_method)
    args.lp_method = int(lp_method)
    sfx = "" if args.lp_method == 1 else f"-m{args.lp_method}"
    args.dataset_prefix = f"{args.data_prefix}/{args.dataset}"
    args.dataset_processed_prefix = f"{args.dataset_prefix}/{args.solver_prefix}inp_tgt{sfx}/"
    args.log_dir = f"{args.log_prefix}/{args.exp_nm}"
    if not args.exist_ok and os.path.exists(args.log_dir):
        k = 2
        while os.path.exists(f"{args.log_dir}{k}"):
            k += 1
        args.log_dir = f"{args.log_dir}{k}"
    args.dev = f"cuda:{args.dev}" if torch.cuda.is_available() else "cpu"
    return args


def parse_args(argv=None):
    return postprocess_args(parser().parse_args(argv))


# ------------------------------------------------------------------- model
def make_model(args, for_eval: bool = False):
    """eval(args.arch) (train.py:79) + --load_from (train.py:80); --fp16 (val.py:269: model.half() after
    the load) only for an evaluation model (``for_eval``): the reference's train.py trains in fp32
    whatever the flag."""
    from .arch import build_model

    model = build_model(args.arch)
    if str(args.load_from).lower() != "none":
        model.load(args.load_from)
    if args.fp16 and for_eval:
        model.half()
    return model.to(args.dev)


def _dist_world():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _average_grads(model, world):
    from .partition import all_reduce_grads

    for p in model.parameters():
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    all_reduce_grads(model)
    for p in model.parameters():
        p.grad.div_(world)


def _partitioned(args, ds, i) -> bool:
    """--partition: graph i of ds takes the row-partitioned path."""
    p = int(getattr(args, "partition", 0))
    return p == 2 or (p == 1 and ds.nnz(i) > args.edge_num_thresh)


def _partition_batch(args, ds, i):
    from .partition import lp_partition_batch

    rank, world = _dist_world()
    return lp_partition_batch(ds.record(i), world, rank, args.dev)


# ------------------------------------------------------------------ run_exp
def run_exp(args, model=None, ds=None):
    """train.py:55-157.  Returns a dict with the per-epoch mean losses, the
    learning rate of every epoch and the checkpoint path."""
    from .train import LOSSES, epoch_batches, make_optimizer
    from .val import accuracy_device

    os.makedirs(args.log_dir, exist_ok=True)
    rank, world = _dist_world()
    replicas = bool(args.replicas) and world > 1
    if replicas and int(getattr(args, "partition", 0)):
        raise ValueError("--replicas and --partition are exclusive (graphs over ranks vs one graph over ranks)")
    if int(getattr(args, "partition", 0)) and args.loss != "balanced":
        raise ValueError("--partition trains with the balanced loss (train.py:39-46, the published experiment)")
    if rank == 0:
        with open(os.path.join(args.log_dir, "args.json"), "w") as fp:
            json.dump({k: v for k, v in vars(args).items() if isinstance(v, (int, float, str, type(None)))}, fp,
                      indent=1)
    if ds is None:
        ds = LPDataset(args.dataset_processed_prefix, thresh_num=args.edge_num_thresh, device=args.dev)
    train_ds, _ = split_train_val(ds, args.seed)
    model = make_model(args) if model is None else model.to(args.dev)
    opt, scheduler = make_optimizer(model, args.opt, args.lr, args.epochs)
    loss_fn = LOSSES[args.loss] if args.loss in LOSSES else None
    if loss_fn is None:
        raise ValueError(f"unknown --loss {args.loss!r} (train.py: balanced / unbalanced / focal)")
    order_rng = torch.Generator().manual_seed(args.seed)  # DataLoader(shuffle=True), same order on every rank
    loss_meter, acc_meter = AverageMeter(), AverageMeter()
    glstep, hist = 0, {"epoch_loss": [], "lr": [], "steps": 0}
    for epoch in range(args.epochs):
        model.train()
        loss_meter.reset(), acc_meter.reset()
        hist["lr"].append(scheduler.get_last_lr()[0])
        order = torch.randperm(len(train_ds), generator=order_rng).tolist()
        if replicas:  # one graph per rank per round; drop the ragged tail (drop_last)
            order = order[: len(order) // world * world][rank::world]
        ep_losses = []
        for idx_graphs, gi in enumerate(order):
            if _partitioned(args, train_ds, gi):
                loss, acc = _partition_train_step(args, model, opt, train_ds, gi)
                glstep += 1
                loss_meter.update(loss)
                ep_losses.append(loss)
                acc_meter.update(acc)
                if glstep % 9 == 1:
                    log.info(f"{epoch} {idx_graphs}/{len(order)} {glstep} {loss_meter.avg:.5f} {acc_meter.avg:.4f} "
                             f"(row-partitioned over {world})")
                continue
            graph = train_ds[gi]
            batches = epoch_batches(graph, args.arch, args.batch_size, dev=args.dev,
                                    seed=args.seed + 1000 * epoch + gi)
            if replicas:
                opt.zero_grad()
            for batch in batches:
                batch.to(args.dev, non_blocking=True)
                glstep += 1
                logit_cons, logit_vars = model(batch)
                logit_cons, logit_vars = logit_cons[:batch.s_bs], logit_vars[:batch.t_bs]
                y_s, y_t = batch.y_s[:batch.s_bs], batch.y_t[:batch.t_bs]
                loss = loss_fn(logit_cons, logit_vars, y_s, y_t)
                assert not torch.isnan(loss).item()  # train.py:126
                if not replicas:
                    opt.zero_grad()
                loss.backward()
                if not replicas:
                    opt.step()
                loss_meter.update(loss.item())
                ep_losses.append(loss.item())
                acc = accuracy_device(torch.cat((logit_cons, logit_vars)).detach(), torch.cat((y_s, y_t)),
                                      logit_cons.shape[0])[0]
                acc_meter.update(acc.item())
                if glstep % 9 == 1:
                    log.info(f"{epoch} {idx_graphs}/{len(order)} {glstep} {loss_meter.avg:.5f} {acc_meter.avg:.4f}")
            if replicas:  # every rank reaches this once per round (same order length on every rank)
                _average_grads(model, world)
                opt.step()
        scheduler.step()  # train.py:153
        hist["epoch_loss"].append(float(np.mean(ep_losses)) if ep_losses else float("nan"))
        hist["steps"] = glstep
        if rank == 0:
            model.save(os.path.join(args.log_dir, "mdl.pth"))  # train.py:154
    if rank == 0:
        model.save(os.path.join(args.log_dir, "mdl.pth"))  # train.py:157
    hist["checkpoint"] = os.path.join(args.log_dir, "mdl.pth")
    return hist


def _partition_train_step(args, model, opt, ds, gi):
    """One full-graph step of graph gi row-partitioned over the ranks (train.py:117-129 on the whole
    graph): forward on every rank's rows, the balanced loss's per-rank shares, backward, one
    all-reduce of the parameter gradients, the optimizer step.  Returns the global (loss, accuracy)."""
    from .partition import _all_reduce_, balanced_distributed, all_reduce_grads, gather_logits
    from .val import accuracy_device

    batch = _partition_batch(args, ds, gi)
    lc, lv = model(batch)
    loss = balanced_distributed(lc, lv, batch.y_s, batch.y_t, batch.n_own)
    opt.zero_grad()
    loss.backward()
    all_reduce_grads(model)
    opt.step()
    tot = _all_reduce_(loss.detach().clone().reshape(1))
    assert not torch.isnan(tot).item()  # train.py:126 (on the whole graph's loss)
    cons, var = gather_logits(lc, lv, batch)
    p = batch.plan
    y = torch.empty(p.m + p.n, dtype=torch.int64, device=cons.device)
    yc, yv = gather_logits(batch.y_s[:, None].float(), batch.y_t[:, None].float(), batch)
    y[:p.m], y[p.m:] = yc[:, 0].long(), yv[:, 0].long()
    acc = accuracy_device(torch.cat((cons, var)), y, p.m)[0]
    return float(tot.item()), float(acc.item())


# --------------------------------------------------------------- validation
@torch.no_grad()
def validation(model, ds, args):
    """val.py:43-68: per graph, model_inference_with_batch (full graph, or
    the every-neighbour k-hop loader above the threshold), then
    accuracy(return_pr=True) on the host; returns (avg_loss = 0, avg_acc)
    and the per-file rows."""
    from .val import accuracy, model_inference_with_batch

    was_training = model.training
    model.eval()
    avg_acc, rows = 0., []
    fp16 = next(model.parameters()).dtype == torch.float16
    for i in range(len(ds)):
        if _partitioned(args, ds, i):  # the whole graph, row-partitioned over the ranks (every rank: all rows)
            from .partition import gather_logits

            batch = _partition_batch(args, ds, i)
            if fp16:  # val.py:269 / utils.py:909-915: fp16 features and edge values, the fp16 partitioned layers
                from .data import batch_to

                batch = batch_to(batch, batch.x_s.device, half=True)
            yl = gather_logits(batch.y_s[:, None].float(), batch.y_t[:, None].float(), batch)
            y = torch.cat(yl)[:, 0].long().cpu()
            lc, lv = gather_logits(*model(batch), batch)
            lc, lv = lc.cpu(), lv.cpu()
        else:
            graph = ds[i]
            lc, lv = model_inference_with_batch(model, graph, args.arch, dev=args.dev, batch_size=args.batch_size,
                                                fp16=fp16)
            y = graph.y if not hasattr(graph, "x_s") else torch.cat((graph.y_s, graph.y_t))
        acc, prec, recl = accuracy(torch.cat((lc, lv), 0), y.cpu(), lc.shape[0], return_pr=True,
                                   dataset_name=args.dataset)
        avg_acc += acc / len(ds)
        rows.append(dict(fn=os.path.basename(ds.path(i)).replace(".pk", ""), acc=float(acc), prec=float(prec),
                         recl=float(recl)))
    if was_training:
        model.train()
    return 0., avg_acc, rows


def main(argv=None):
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(message)s")
    args = parse_args(argv)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env > 1 and not (args.replicas or args.partition):
        # under a launcher without --replicas / --partition every rank would train the full schedule on
        # its own and write args.json / mdl.pth into the same directory: refuse instead
        raise SystemExit(f"WORLD_SIZE={world_env}: pass --replicas 1 for data-parallel training over graphs, "
                         "--partition 1 to row-partition the large graphs over the ranks (or run one process)")
    if args.replicas or args.partition:
        import torch.distributed as dist

        if world_env > 1 and not dist.is_initialized():
            backend = "nccl" if torch.cuda.is_available() else "gloo"
            if torch.cuda.is_available():  # the rank's GPU first: RCCL binds its communicator to the current device
                args.dev = f"cuda:{int(os.environ.get('LOCAL_RANK', '0'))}"
                torch.cuda.set_device(args.dev)
            dist.init_process_group(backend, device_id=torch.device(args.dev) if backend == "nccl" else None)
    if args.phase == "train":
        hist = run_exp(args)
        print(json.dumps({"epoch_loss": hist["epoch_loss"], "checkpoint": hist["checkpoint"]}))
        return 0
    ds = LPDataset(args.dataset_processed_prefix, thresh_num=args.edge_num_thresh, device=args.dev)
    _, val_ds = split_train_val(ds, args.seed)
    eval_ds = ds if args.split == "trainval" else val_ds
    model = make_model(args, for_eval=True)
    _, avg_acc, rows = validation(model, eval_ds, args)
    print(json.dumps({"avg_acc": avg_acc, "graphs": rows}))
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Multi-process data-parallel path on CPU (gloo, world_size 2).

1. Coordinate sharding (configs M/C1-C3 on N GPUs): each rank fits its contiguous row block of
   the grid; one summed gradient all-reduce per step (GradAllReducer(op='sum')) makes the
   sharded run reproduce the single-process full-grid fit exactly (SSE loss).
2. train_ddp with a DistributedSampler (configs 4/5): averaged gradients (DDP semantics), ranks
   stay bit-identical, only rank 0 writes checkpoints.
The model is the CPU oracle (the SIREN kernels need a GPU); what is under test is the host-side
exchange logic, which is device-independent.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import siren_oracle as orc


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def sse(out, gt):
    return {"img_loss": ((out["model_out"] - gt["img"]) ** 2).sum() / (128 * 128)}


def _sharded_worker(rank, world, port, side, steps, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    from siren_mri_amd.training_ddp import ddp_setup, shard_rows, GradAllReducer
    ddp_setup(rank, world, backend="gloo")
    torch.manual_seed(rank + 100)  # deliberately different local init: the broadcast must fix it
    model = orc.OracleSiren(hidden_features=32, num_hidden_layers=1, seed=rank + 7)
    reducer = GradAllReducer(model.parameters(), op="sum")
    coords = orc.get_mgrid(side)
    img = torch.sin(3 * coords[:, :1]) * torch.cos(2 * coords[:, 1:])
    lo, hi = shard_rows(coords.shape[0], rank, world)
    inp = {"coords": coords[lo:hi][None]}
    gt = {"img": img[lo:hi][None]}
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters())
    for _ in range(steps):
        loss = sse(model(inp), gt)["img_loss"]
        loss.backward()
        reducer()
        opt.step()
        opt.zero_grad()
    out_q.put((rank, [p.detach().numpy().copy() for p in model.parameters()]))
    dist.barrier()
    dist.destroy_process_group()


def test_coordinate_sharded_fit_equals_full_fit():
    world, side, steps = 2, 16, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, side, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference: rank 0's init (broadcast) on the full grid
    model = orc.OracleSiren(hidden_features=32, num_hidden_layers=1, seed=7)
    coords = orc.get_mgrid(side)
    img = torch.sin(3 * coords[:, :1]) * torch.cos(2 * coords[:, 1:])
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters())
    for _ in range(steps):
        loss = sse(model({"coords": coords[None]}), {"img": img[None]})["img_loss"]
        loss.backward()
        opt.step()
        opt.zero_grad()
    for a, b in zip(results[0], results[1]):
        assert np.array_equal(a, b), "ranks diverged"
    for a, ref in zip(results[0], model.parameters()):
        assert orc.norm_rel(torch.from_numpy(a), ref.detach()) < 1e-5


class _SliceSet(torch.utils.data.Dataset):
    def __init__(self, n=8, side=8):
        self.coords = orc.get_mgrid(side)
        g = torch.Generator().manual_seed(0)
        self.imgs = [torch.randn(side * side, 1, generator=g) for _ in range(n)]

    def __len__(self):
        return len(self.imgs)

    def __getitem__(self, i):
        return {"coords": self.coords}, {"img": self.imgs[i]}


def _train_ddp_worker(rank, world, port, root, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    from siren_mri_amd import training_ddp
    training_ddp.ddp_setup(rank, world, backend="gloo")
    model = orc.OracleSiren(hidden_features=16, num_hidden_layers=1, seed=rank)
    ds = _SliceSet()
    sampler = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True)
    loader = torch.utils.data.DataLoader(ds, batch_size=2, sampler=sampler)
    training_ddp.train_ddp(model, loader, epochs=2, lr=1e-3, steps_til_summary=1000, epochs_til_checkpoint=1000,
                           model_dir=root, loss_fn=sse, summary_fn=lambda *a, **k: None, device=rank,
                           clip_grad=True)
    out_q.put((rank, [p.detach().numpy().copy() for p in model.parameters()]))
    dist.barrier()
    dist.destroy_process_group()


def test_train_ddp_ranks_stay_identical(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    root = str(tmp_path / "ddp_run")
    procs = [ctx.Process(target=_train_ddp_worker, args=(r, world, port, root, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for a, b in zip(results[0], results[1]):
        assert np.array_equal(a, b)
    assert os.path.exists(os.path.join(root, "checkpoints", "model_final.pth"))
    losses = np.loadtxt(os.path.join(root, "checkpoints", "train_losses_final.txt"))
    assert losses.shape == (4,)  # 2 epochs x 2 local batches of 2 slices


def test_shard_rows_partition():
    from siren_mri_amd.training_ddp import shard_rows
    n, world = 262144 + 3, 8
    spans = [shard_rows(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


def _rank_batches(rank, n=4, side=8):
    coords = orc.get_mgrid(side)
    g = torch.Generator().manual_seed(1000 + rank)
    return [({"coords": coords[None]}, {"img": torch.randn(1, side * side, 1, generator=g)}) for _ in range(n)]


def _accum_worker(rank, world, port, op, clip, root, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    from siren_mri_amd import training_ddp
    training_ddp.ddp_setup(rank, world, backend="gloo")
    model = orc.OracleSiren(hidden_features=16, num_hidden_layers=1, seed=3)
    training_ddp.train_ddp(model, _rank_batches(rank), epochs=1, lr=1e-3, steps_til_summary=1000,
                           epochs_til_checkpoint=1000, model_dir=root, loss_fn=sse,
                           summary_fn=lambda *a, **k: None, device=rank, clip_grad=clip,
                           accumulation_steps=2, grad_op=op)
    out_q.put((rank, [p.detach().numpy().copy() for p in model.parameters()]))
    dist.barrier()
    dist.destroy_process_group()


def _accum_reference(world, op, clip, acc=2):
    """Single-process statement of the intended semantics (training_ddp.py:96-109 with DDP
    averaging, or a sum for coordinate-sharded fits): every micro-step's gradient is reduced over
    ranks exactly once, added to the window's gradient, and clipped every micro-step."""
    from siren_mri_amd.training import make_adam
    model = orc.OracleSiren(hidden_features=16, num_hidden_layers=1, seed=3)
    params = list(model.parameters())
    optim = make_adam(params, 1e-3)
    batches = [_rank_batches(r) for r in range(world)]
    for step in range(len(batches[0])):
        per_rank = []
        for r in range(world):
            inp, gt = batches[r][step]
            loss = sse(model(inp), gt)["img_loss"].mean() / acc
            per_rank.append(torch.autograd.grad(loss, params))
        with torch.no_grad():
            for i, p in enumerate(params):
                red = sum(g[i] for g in per_rank)
                if op == "mean":
                    red = red / world
                p.grad = red.clone() if p.grad is None else p.grad + red
        if clip:
            torch.nn.utils.clip_grad_norm_(params, max_norm=1.0)
        if (step + 1) % acc == 0:
            optim.step()
            optim.zero_grad()
    return [p.detach().numpy() for p in params]


@pytest.mark.parametrize("op", ["sum", "mean"])
@pytest.mark.parametrize("clip", [False, True])
def test_grad_accumulation_reduces_each_micro_step_once(tmp_path, op, clip):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    root = str(tmp_path / "acc_run")
    procs = [ctx.Process(target=_accum_worker, args=(r, world, port, op, clip, root, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _accum_reference(world, op, clip)
    for a, b in zip(results[0], results[1]):
        assert np.array_equal(a, b), "ranks diverged"
    for a, r in zip(results[0], ref):
        assert orc.norm_rel(torch.from_numpy(a), torch.from_numpy(r)) < 1e-5


def test_model_dir_not_deleted_without_consent(tmp_path, monkeypatch):
    import io
    from siren_mri_amd.training import prepare_model_dir
    d = tmp_path / "exp"
    (d / "checkpoints").mkdir(parents=True)
    (d / "checkpoints" / "model_final.pth").write_bytes(b"keep")
    monkeypatch.setattr("sys.stdin", io.StringIO(""))  # not a TTY (nohup / batch / pipe)
    with pytest.raises(FileExistsError):
        prepare_model_dir(str(d))
    assert (d / "checkpoints" / "model_final.pth").read_bytes() == b"keep"
    prepare_model_dir(str(d), overwrite=True)
    assert not (d / "checkpoints" / "model_final.pth").exists()


def _overlap_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    from siren_mri_amd.training_ddp import ddp_setup, GradAllReducer
    ddp_setup(rank, world, backend="gloo")
    model = orc.OracleSiren(hidden_features=32, num_hidden_layers=2, seed=rank + 1)
    # ~4 KB buckets: several buckets, so the early (top-layer) ones launch from the hooks
    red = GradAllReducer(model.parameters(), op="mean", bucket_bytes=4096)
    coords = orc.get_mgrid(8)[None] * (1 + rank)
    launched_during_backward = []
    for step in range(2):
        red.begin()
        loss = model({"coords": coords})["model_out"].square().sum()
        loss.backward()
        launched_during_backward.append(sum(w is not None for w in red._work))
        red()
        grads = [p.grad.detach().clone() for p in model.parameters()]
        in_slots = all(any(p.grad.data_ptr() == v.data_ptr() for v in [red._views[p]]) for p in model.parameters())
        # the reference: average of both ranks' gradients of the same (broadcast) parameters
        ref = []
        for r in range(world):
            m2 = orc.OracleSiren(hidden_features=32, num_hidden_layers=2, seed=0)
            m2.load_state_dict(model.state_dict())
            m2({"coords": orc.get_mgrid(8)[None] * (1 + r)})["model_out"].square().sum().backward()
            ref.append([p.grad for p in m2.parameters()])
        err = max(orc.norm_rel(g, (a + b) / 2) for g, a, b in zip(grads, ref[0], ref[1]))
        with torch.no_grad():
            for p in model.parameters():
                p -= 1e-3 * p.grad
        model.zero_grad(set_to_none=True)
    out_q.put((rank, len(red.buckets), launched_during_backward, in_slots, err))
    dist.barrier()
    dist.destroy_process_group()


def test_bucketed_allreduce_overlaps_backward_without_copies():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r[0], r[1:]) for r in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for nb, launched, in_slots, err in res.values():
        assert nb > 2
        assert all(k == nb for k in launched), launched  # every bucket launched from the hooks
        assert in_slots
        assert err < 1e-6

"""GPU: siren_mri_amd.optim.Adam (one native launch) against torch.optim.Adam's default foreach
path (the reference's optimizer, training.py:29) — same operation order; the two compilers'
multiply-add contraction differs, so values agree to an ulp (rtol 1e-6), not bit for bit."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("kw", [dict(), dict(weight_decay=0.01), dict(maximize=True, betas=(0.8, 0.99))])
def test_adam_matches_torch_foreach(kw):
    from siren_mri_amd.optim import Adam
    g = torch.Generator().manual_seed(0)
    shapes = [(256, 2), (256,), (256, 256), (256,), (1, 256), (1,)]
    init = [torch.randn(s, generator=g) for s in shapes]
    ours = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    ref = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    o1 = Adam(ours, lr=1e-3, **kw)
    o2 = torch.optim.Adam(ref, lr=1e-3, foreach=True, **kw)
    for step in range(7):
        grads = [torch.randn(s, generator=g).to(DEV) for s in shapes]
        for p, q, gr in zip(ours, ref, grads):
            p.grad = gr.clone()
            q.grad = gr.clone()
        o1.step()
        o2.step()
    torch.cuda.synchronize()
    for p, q in zip(ours, ref):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(o1.state[p]["exp_avg"], o2.state[q]["exp_avg"], rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(o1.state[p]["exp_avg_sq"], o2.state[q]["exp_avg_sq"], rtol=1e-6, atol=1e-10)
        assert float(o1.state[p]["step"]) == float(o2.state[q]["step"])


def test_adam_state_dict_round_trip_with_torch():
    from siren_mri_amd.optim import Adam
    p = torch.nn.Parameter(torch.randn(10, device=DEV))
    o1 = Adam([p], lr=1e-2)
    p.grad = torch.randn(10, device=DEV)
    o1.step()
    o2 = torch.optim.Adam([p], lr=1e-2)
    o2.load_state_dict(o1.state_dict())
    assert torch.equal(o2.state[p]["exp_avg"], o1.state[p]["exp_avg"])


@pytest.mark.parametrize("form", ["table", "computed"])
@pytest.mark.parametrize("sizes", [(300,), (300000, 77, 256 * 256), tuple(range(1, 60))])
def test_adam_graph_mode_replay_matches_eager(sizes, form, monkeypatch):
    """enable_graph_mode(): bias corrections from device step counters, so a hipGraph of the
    step replays with the right t each time (same values as eager steps). Table form: one launch
    per chunk of tensors, its workgroups advancing their own counters (59 tensors: two
    chunks); computed form (a table too long for the betas): a single-thread launch per step
    advances the group counter and computes the scalars."""
    from siren_mri_amd.optim import Adam
    if form == "computed":
        monkeypatch.setattr(Adam, "_TABLE_MAX", 4)
    g = torch.Generator().manual_seed(1)
    inits = [torch.randn(n, generator=g) for n in sizes]
    grads = [[torch.randn(n, generator=g).to(DEV) for n in sizes] for _ in range(6)]
    p_e = [torch.nn.Parameter(t.clone().to(DEV)) for t in inits]
    o_e = Adam(p_e, lr=1e-2)
    for gs in grads:
        for p, gr in zip(p_e, gs):
            p.grad = gr.clone()
        o_e.step()
    p_g = [torch.nn.Parameter(t.clone().to(DEV)) for t in inits]
    o_g = Adam(p_g, lr=1e-2)
    o_g.enable_graph_mode()
    gbuf = [torch.empty(n, device=DEV) for n in sizes]
    for p, b, gr in zip(p_g, gbuf, grads[0]):
        p.grad = b
        b.copy_(gr)
    o_g.step()  # eager first step creates the device counter (t = 1)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        o_g.step()
    for gs in grads[1:]:
        for b, gr in zip(gbuf, gs):
            b.copy_(gr)
        graph.replay()
    torch.cuda.synchronize()
    for a, b in zip(p_g, p_e):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-6, atol=1e-7)
    o_g.sync_graph_steps()
    # the capture itself does not step: 1 eager + 5 replays = 6 steps, like the eager optimizer
    assert float(o_g.state[p_g[0]]["step"]) == 6.0


def test_adam_graph_mode_lr_schedule_rewrites_table_in_place():
    """an lr change in graph mode rewrites the step-scalar table in place (its length
    depends on the betas only): nothing is retired or allocated per lr value, and a hipGraph
    captured before the change replays the NEW lr, as the eager optimizer does."""
    from siren_mri_amd.optim import Adam
    g = torch.Generator().manual_seed(2)
    init = torch.randn(4096, generator=g)
    grads = [torch.randn(4096, generator=g).to(DEV) for _ in range(6)]
    lrs = [1e-2, 1e-2, 5e-3, 2.5e-3, 1e-3, 1e-3]
    p_e = torch.nn.Parameter(init.clone().to(DEV))
    o_e = Adam([p_e], lr=lrs[0])
    for lr, gr in zip(lrs, grads):
        o_e.param_groups[0]["lr"] = lr
        p_e.grad = gr.clone()
        o_e.step()
    p_g = torch.nn.Parameter(init.clone().to(DEV))
    o_g = Adam([p_g], lr=lrs[0])
    o_g.enable_graph_mode()
    buf = torch.empty(4096, device=DEV)
    p_g.grad = buf
    buf.copy_(grads[0])
    o_g.step()
    table = o_g._tables[id(o_g.param_groups[0])][2]
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        o_g.step()
    for lr, gr in zip(lrs[1:], grads[1:]):
        o_g.param_groups[0]["lr"] = lr  # a scheduler's per-step lr
        o_g.update_graph_scalars()
        buf.copy_(gr)
        graph.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(p_g.detach(), p_e.detach(), rtol=1e-6, atol=1e-7)
    assert o_g._tables[id(o_g.param_groups[0])][2] is table
    assert not o_g.__dict__.get("_retired")

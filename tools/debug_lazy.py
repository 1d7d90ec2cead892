import sys, torch
sys.path.insert(0, '.')
import __graft_entry__ as g
asme = g.load_package()
dev = torch.device('cuda:0')
def run(V, D, steps, idfun, lazy):
    torch.manual_seed(0)
    base = torch.randn(V, D, device=dev)
    p = torch.nn.Parameter(base.clone()); p._asme_table_grad = asme.ops.TableGrad()
    opt = asme.FusedAdam([p], lr=3e-3, betas=(0.99, 0.998), weight_decay=1e-3, lazy_table=lazy)
    mp = torch.full((V,), -1, dtype=torch.int32, device=dev)
    gen = torch.Generator(device=dev).manual_seed(1)
    for s in range(steps):
        ids = idfun(s).to(dev)
        rows = torch.randn(ids.numel(), D, device=dev, generator=gen)
        plan = asme.ops.SparseTablePlan(p, [ids], mp)
        asme._lib.call("asme_scatter_add_rows", rows.data_ptr(), plan.inverse_of(ids).data_ptr(), ids.numel(), D,
                       plan.grad_rows.data_ptr(), plan.capacity, 1.0, asme._lib.stream())
        p._asme_table_grad.plan = plan
        opt.step()
    opt.flush()
    return p.detach().clone()
V, D = 64, 64
cases = {
 'all rows every step': lambda s: torch.arange(V),
 'row 0 only': lambda s: torch.tensor([0]),
 'none touched after step0': lambda s: torch.arange(V) if s == 0 else torch.tensor([0]),
}
for name, f in cases.items():
    for steps in (1, 2, 3):
        a, b = run(V, D, steps, f, True), run(V, D, steps, f, False)
        diff = (a != b)
        print(f"{name:28s} steps={steps} ndiff={int(diff.sum())} maxabs={float((a-b).abs().max()):.3e}",
              'rows', diff.any(1).nonzero().flatten()[:8].tolist())

import sys, math, torch, torch.nn.functional as F
sys.path.insert(0, '.')
import __graft_entry__ as g
asme = g.load_package()
torch.manual_seed(0)
dev = torch.device('cuda:0')
for (B, H, L, dk, causal) in [(1, 1, 16, 16, False), (1, 1, 16, 16, True), (2, 2, 40, 64, True)]:
    D = H * dk
    qkv = torch.randn(B, L, 3 * D)
    gr = torch.randn(B, L, D)
    x = qkv.clone().requires_grad_(True)
    q, k, v = [x[..., i * D:(i + 1) * D].view(B, L, H, dk).transpose(1, 2) for i in range(3)]
    s = q @ k.transpose(-2, -1) / math.sqrt(dk)
    if causal:
        s = s.masked_fill(torch.tril(torch.ones(L, L)) == 0, -1e9)
    o = (F.softmax(s, -1) @ v).transpose(1, 2).reshape(B, L, D)
    o.backward(gr)
    xd = qkv.to(dev).requires_grad_(True)
    od = asme.ops.attention(xd, None, H, causal, 0.0)
    od.backward(gr.to(dev))
    gd = xd.grad.cpu()
    for i, nm in enumerate('qkv'):
        a, b = gd[..., i * D:(i + 1) * D], x.grad[..., i * D:(i + 1) * D]
        print(B, H, L, dk, causal, nm, 'relerr', float((a - b).abs().max() / b.abs().max()))
    if L == 16 and not causal:
        print('dq ref', x.grad[0, :4, :4]); print('dq got', gd[0, :4, :4])
        print('dv ref', x.grad[0, :4, 2*D:2*D+4]); print('dv got', gd[0, :4, 2*D:2*D+4])

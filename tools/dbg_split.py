import sys, math, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from fsp_amd import ops, _native as N
from test_split_w16_gpu import split_form, _w16
dev = torch.device('cuda')
g = torch.Generator(device="cpu").manual_seed(301)
M, W = 300, 512
x = (torch.randn(M, W, generator=g) + 0.5 * torch.randn(M, 1, generator=g)).to(dev)
wfc = _w16((4 * W, W), g, 1 / math.sqrt(W)).to(dev)
bfc = ops.split_pack(wfc)
bias = torch.randn(4 * W, generator=g).to(dev)
for e in (N.EPI_BIAS_QGELU | N.QGELU_DERIV, N.EPI_BIAS_QGELU):
    y, d = ops.gemm(x, bfc, e, bias=bias, want_out2=True)
    ys, ds = ops.gemm(x, bfc, e | N.OUT_SPLIT, bias=bias, want_out2=True)
    a = ys.view(torch.int32); b = split_form(y).view(torch.int32)
    bad = (a != b).nonzero()
    print(hex(e), 'mismatch', bad.shape[0], 'of', a.numel())
    if bad.shape[0]:
        r, c = bad[0].tolist()
        print(' first', r, c)
        gh = ys[r].view(torch.float16); th = split_form(y)[r].view(torch.float16)
        cc = c * 2
        print(' gpu halfs', gh[cc-4:cc+6].tolist())
        print(' ref halfs', th[cc-4:cc+6].tolist())
        grp = (c * 2) // 16
        print(' y group', y[r, grp*8:grp*8+8].tolist())
        print(' cols with mismatch (first 20):', sorted(set((bad[:, 1] % 8).tolist()))[:20], 'rows', bad[:, 0].unique().numel())

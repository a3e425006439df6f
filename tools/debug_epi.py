"""Which output of the staged-epilogue A/B differs, and where (debug aid)."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, os.path.join(REPO, 'tests'))
import torch  # noqa: E402
from test_gpu_kernels import _nhwc  # noqa: E402
from eegan_hip import functional as Fn  # noqa: E402

gpu = torch.device('cuda', 0)
os.environ['EEGAN_CONV_TARGET'] = sys.argv[1] if len(sys.argv) > 1 else '1'
N, Cin, H, W, Cout, k, st, pad = 2, 48, 32, 32, 32, 3, 1, 1
torch.manual_seed(N * Cin + Cout + H)
g = Fn.Geom(Cout, k, k, st, pad, pad, 0)
x = _nhwc(torch.randn(N, Cin, H, W), gpu)
Wt = (torch.randn(Cout, Cin, k, k) * 0.05).to(gpu)
b = torch.randn(Cout).to(gpu)
gam = torch.tensor([0.7]).to(gpu)
Ho, Wo = g.out_hw(H, W)
res = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
dz = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
gate = _nhwc(torch.randn(N, Cin, H, W), gpu)
halfres = _nhwc(torch.randn(N, Cin, H // 2, W // 2), gpu)
lrelu = Fn.ACT_CODES['lrelu']
outs = []
for on in ('0', '1'):
    os.environ['EEGAN_CONV_STAGE_EPI'] = on
    outs.append([Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu, res=res, gamma=gam).float().cpu(),
                 Fn.conv_fwd_raw(x, Wt, None, g).float().cpu(),
                 Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape)).float().cpu(),
                 Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), gate=gate, gate_act=lrelu).float().cpu(),
                 Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), res=halfres, res_up2=1, res_scale=0.25).float().cpu()])
for i, (a, c) in enumerate(zip(*outs)):
    d = (a - c).abs()
    print(i, tuple(a.shape), 'equal' if torch.equal(a, c) else 'DIFF max %g at %s, count %d' % (
        d.max().item(), tuple(int(v) for v in (d == d.max()).nonzero()[0]), int((d > 0).sum())))
    if not torch.equal(a, c):
        nz = (d > 0).nonzero()
        print('   channels', sorted(set(nz[:, 1].tolist()))[:20], 'rows', sorted(set(nz[:, 2].tolist()))[:20],
              'cols', sorted(set(nz[:, 3].tolist()))[:20])

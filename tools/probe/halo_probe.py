"""Driver of tools/probe/halo_probe.hip (diagnostic): the halo-tile 3x3 conv
prototype against the library's conv (Fn.conv_fwd_raw / conv_bwd_data_raw) on
the same packed weights -- agreement and HIP-event timing per shape."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
import torch  # noqa: E402

SHAPES = [  # N, C, H, W, K
    (16, 128, 64, 64, 128), (16, 64, 128, 128, 64), (32, 64, 128, 128, 64), (32, 128, 64, 64, 128),
    (32, 256, 32, 32, 256), (16, 256, 32, 32, 256), (16, 64, 64, 64, 64), (16, 128, 128, 128, 64),
]


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    from eegan_hip import functional as Fn
    from eegan_hip.tensor import empty_nhwc, ld_of, stream
    lib = ctypes.CDLL(os.path.join(REPO, 'tools', 'probe', 'halo_probe.so'))
    P = ctypes.c_void_p
    I = ctypes.c_int
    lib.halo_conv.argtypes = [I, I, P, P, P, P] + [I] * 10 + [ctypes.c_float, ctypes.c_long, ctypes.c_long, I, P]
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else '0,1,2,3').split(',')]
    knocks = [int(k) for k in (sys.argv[2] if len(sys.argv) > 2 else '0').split(',')]
    shapes = SHAPES if len(sys.argv) <= 3 else [SHAPES[int(i)] for i in sys.argv[3].split(',')]
    for (N, C, H, W, K) in shapes:
        x = Fn.to_nhwc_bf16(torch.randn(N, C, H, W, device=dev))
        Wt = (torch.randn(K, C, 3, 3, device=dev) * (1.0 / (9 * C) ** 0.5)).contiguous(memory_format=torch.channels_last)
        b = torch.randn(K, device=dev) * 0.1
        g = Fn.Geom(K, 3, 3, 1, 1, 1, 0)
        flops = 2.0 * N * H * W * K * C * 9
        for mode in (0, 1):
            if mode == 0:
                ref = Fn.conv_fwd_raw(x, Wt, b, g)
                wp = Fn.pack_weight(Wt, False)
                src, Cin, Kout = x, C, K
                tref = timeit(lambda: Fn.conv_fwd_raw(x, Wt, b, g))
            else:
                dz = Fn.to_nhwc_bf16(torch.randn(N, K, H, W, device=dev))
                ref = Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape))
                wp = Fn.pack_weight(Wt, True)
                src, Cin, Kout = dz, K, C
                tref = timeit(lambda: Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape)))
            cgp = (Cin + 31) // 32 * 32
            kw = (9 * cgp + 31) // 32 * 32
            line = '%-22s %s ref %7.2f us %6.1f TF' % ((N, C, H, W, K), 'fwd ' if mode == 0 else 'bwdd',
                                                     tref, flops / tref / 1e6)
            for v, kn in [(v, k) for v in variants for k in knocks]:
                out = empty_nhwc(N, Kout, H, W, dev)
                bias = b if mode == 0 else None

                def run():
                    return lib.halo_conv(v, mode, src.data_ptr(), wp.data_ptr(), bias.data_ptr() if bias is not None
                                         else None, out.data_ptr(), N, H, W, ld_of(src), Cin, cgp, Kout, kw,
                                         ld_of(out), 0, 0.2, src.numel() * 2 if src.is_contiguous() else
                                         N * H * W * ld_of(src) * 2, wp.numel() * 2, kn, stream())
                rc = run()
                if rc:
                    line += ' | v%d n/a' % v
                    continue
                torch.cuda.synchronize()
                err = float((out.float() - ref.float()).norm() / ref.float().norm()) if kn == 0 else 0.0
                t = timeit(run)
                line += ' | v%d/k%d %7.2f us %6.1f TF err %.1e' % (v, kn, t, flops / t / 1e6, err)
            print(line, flush=True)


if __name__ == '__main__':
    main()

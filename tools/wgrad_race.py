"""Where a non-deterministic row-blocked weight gradient goes wrong (diagnostic, GPU).

  python tools/wgrad_race.py [B] [Cin] [Cout] [H] [K] [scaled] [reps]

Runs the row-blocked wgrad `reps` times on one set of operands, compares each result with the gather
wgrad (kernel_off bit 2) at the fp32 bar, and prints, per bad run, how many weights are off and how
they spread over output rows m (by 32-row wave), input columns j, kernel rows kh and taps kw."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

DEV = torch.device("cuda", 0)


def main(B=8, Cin=96, Cout=96, H=64, K=3, scaled=1, reps=20):
    import gan_amd  # noqa: F401
    from gan_amd import ops
    geo = ops.conv_geo(B, Cin, H, H, Cout, K, 1, (K - 1) // 2, 1)
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(Cin, B, H, H, generator=g, device=DEV)
    gy = torch.randn(Cout, B, H, H, generator=g, device=DEV)
    sx = torch.rand(Cin, B, generator=g, device=DEV) + 0.5 if scaled else None
    sy = torch.rand(Cout, B, generator=g, device=DEV) + 0.5 if scaled else None
    with ops.patch_conv(3):
        ref = ops._conv_wgrad(geo, x, gy, sx, sy, 1.0)
    scale = ref.abs().max()
    nbad_runs = 0
    for r in range(reps):
        got = ops._conv_wgrad(geo, x, gy, sx, sy, 1.0)
        torch.cuda.synchronize()
        bad = (got - ref).abs() > 1e-4 * scale
        n = int(bad.sum())
        if n == 0:
            continue
        nbad_runs += 1
        idx = bad.nonzero()
        m, j, kh, kw = idx[:, 0], idx[:, 1], idx[:, 2], idx[:, 3]
        hist = lambda t, n: torch.bincount(t, minlength=n).tolist()      # noqa: E731
        print(f"run {r}: {n} bad of {ref.numel()}, max |d| {float((got - ref).abs().max()):.3g}", flush=True)
        print("   by m//32:", hist(m // 32, (Cout + 31) // 32), " by j//32:", hist(j // 32, (Cin + 31) // 32),
              " by kh:", hist(kh, K), " by kw:", hist(kw, K), flush=True)
        print("   by m%32:", hist(m % 32, 32), flush=True)
        print("   by j%32:", hist(j % 32, 32), flush=True)
    print(f"{nbad_runs} of {reps} runs off", flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])

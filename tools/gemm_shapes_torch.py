"""Vendor-library reference point for the prefill GEMM shapes: torch.nn.functional.linear (bf16,
hipBLASLt on ROCm) on bloom-1b1 / 3b / 7b1 prefill projections, device time per call from HIP
events over hipGraph replays of 20 back-to-back calls.  A measurement aid for DESIGN.md (what the library reaches on
the same M = 512 shapes our gemm_mfma2_kernel runs), not part of the product path.

    python tools/gemm_shapes_torch.py [M]
"""
import sys

import torch
import torch.nn.functional as F

PEAK = 2.5e15  # dense bf16 MFMA peak, MI355X_MICROARCH.md


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    dev = torch.device("cuda:0")
    shapes = {"bloom-1b1": 1536, "bloom-3b": 2560, "bloom-7b1": 4096}
    tot_flop, tot_s = 0.0, 0.0
    for name, h in shapes.items():
        for what, n, k in (("qkv", 3 * h, h), ("dense", h, h), ("fc1", 4 * h, h), ("fc2", h, 4 * h)):
            x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
            w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02
            b = torch.randn(n, device=dev, dtype=torch.bfloat16)
            for _ in range(20):
                F.linear(x, w, b)
            torch.cuda.synchronize()
            # captured in a graph: host launch cost (~10-20 us per F.linear call) would otherwise
            # be what the events measure at these sizes
            per, reps = 20, 20
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            with torch.cuda.stream(side):
                with torch.cuda.graph(g, stream=side):
                    for _ in range(per):
                        F.linear(x, w, b)
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            s = e0.elapsed_time(e1) / 1e3 / (reps * per)
            flop = 2.0 * M * n * k
            if name == "bloom-1b1":
                tot_flop += flop
                tot_s += s
            print(f"{name:9s} {what:5s} M={M} N={n:5d} K={k:5d}: {s * 1e6:8.2f} us  {flop / s / 1e12:7.1f} TFLOP/s  "
                  f"frac {flop / s / PEAK:.3f}", flush=True)
    print(f"bloom-1b1 layer (4 GEMMs) M={M}: {tot_s * 1e6:.1f} us, {tot_flop / tot_s / 1e12:.1f} TFLOP/s, "
          f"frac {tot_flop / tot_s / PEAK:.3f}", flush=True)


if __name__ == "__main__":
    main()

"""Time the ResNet-152 ID classifier forward on a frame's 32 boxes (random weights), for rocprof."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"))


def main():
    import torch
    from mqhip.resnet_id import ResNetIdHip, make_random_weights
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    m = ResNetIdHip(make_random_weights(152, seed=0), depth=152)
    x = torch.randn((n, 224, 224, 3), device="cuda").to(torch.bfloat16)
    for _ in range(3):
        m.forward(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        m.forward(x)
    torch.cuda.synchronize()
    print(f"ResNet-152 ID forward, {n} boxes: {(time.perf_counter() - t0) * 100:.2f} ms", flush=True)


if __name__ == "__main__":
    main()

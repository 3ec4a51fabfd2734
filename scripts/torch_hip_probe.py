"""Does torch's HIP runtime coexist with libksa_gpu.so in one process, in either init order?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

order = sys.argv[1]
if order == "ksa-before-import":  # our library loaded and used before torch is even imported
    from kube_sqs_autoscaler_amd.ops import gpu

    print(order, "ksa devices", gpu.device_count(), flush=True)
    import torch

    print(order, "torch available", torch.cuda.is_available(), torch.cuda.device_count(), flush=True)
    sys.exit(0)
import torch  # noqa: E402

from kube_sqs_autoscaler_amd.ops import gpu  # noqa: E402

if order == "torch-first":
    torch.cuda.set_device(0)
    x = torch.ones(4, device="cuda").sum().item()
    n = gpu.device_count()
    print(order, "torch ok", x, "ksa devices", n, flush=True)
else:
    n = gpu.device_count()
    print(order, "ksa devices", n, flush=True)
    print("torch available", torch.cuda.is_available(), torch.cuda.device_count(), flush=True)
    torch.cuda.set_device(0)
    print(order, "torch ok", torch.ones(4, device="cuda").sum().item(), flush=True)

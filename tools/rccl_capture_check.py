"""Does an RCCL collective through torch.distributed capture into a hipGraph and
replay correctly?  One process, a world of one (nccl backend = RCCL on ROCm):
all_reduce and all_gather_into_tensor captured with a kernel either side, the
graph replayed on new inputs, results checked.  Prints one JSON line.
  python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \\
      --master-port 29511 tools/rccl_capture_check.py"""
import json

import torch
import torch.distributed as dist


def main():
    dist.init_process_group("nccl")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {}
    x = torch.randn(1 << 20, device=dev)
    y = torch.empty(1 << 20, device=dev)
    g_out = torch.empty(1 << 20, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm the communicator outside capture
        for _ in range(3):
            y.copy_(x * 2.0)
            dist.all_reduce(y)
            dist.all_gather_into_tensor(g_out, y)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            y.copy_(x * 2.0)
            dist.all_reduce(y)
            dist.all_gather_into_tensor(g_out, y)
            g_out.mul_(0.5)
        for trial in range(3):
            x.normal_()
            g.replay()
            torch.cuda.synchronize()
            ok = torch.allclose(g_out, x, rtol=0, atol=1e-6)
            out["replay%d" % trial] = bool(ok)
        out["captured"] = True
    except Exception as e:  # noqa: BLE001
        out["captured"] = False
        out["error"] = repr(e)[:300]
    print(json.dumps(out))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

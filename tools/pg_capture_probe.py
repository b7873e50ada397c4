"""Reproduce (or rule out) the ProcessGroupNCCL watchdog abort seen once in ~10 round-5 GPU suites:
"operation not permitted on an event last recorded in a capturing stream" (graphs.StepGraph).

Hypothesis: the watchdog still holds an EAGER work of process group G (its end event recorded on
G's internal RCCL stream) when a captured collective on G makes that same internal stream join
the graph capture.  HIP then refuses hipEventQuery on the eager event (its recording stream is
capturing), the watchdog rethrows, the process aborts.  Nothing about the event itself is
captured -- the stream it was recorded on is.

    python tools/pg_capture_probe.py MODE

MODE (every mode: 4 eager all-reduces on group G, then a capture held open for 1.5 s that holds
one all-reduce):
  twin      eager works issued from the capture stream s, captured work on a fresh group
  hazard    eager works issued from s, captured work on G
  estream   eager works issued from another stream E, captured work on G (from s)
  async     eager works issued from s with async_op=True (+ wait), captured work on G
  product   the product's layout (dist.dedicated_stream): eager SyncBN-like all-reduces on the
            "eager" stream and a GradBuckets flush on "bucket_eager", then a capture on the
            "capture" stream holding the same collectives (GradBuckets on "bucket_capture")

Round 6 result: `twin` ABORTS (so the first hypothesis above is wrong: the group does not
matter).  The test of the second hypothesis: a blocking (async_op=False) collective runs on the
CURRENT stream and records its end event there; the watchdog aborts when that stream is capturing
when it polls the eager work.  Then `estream` and `async` pass -- and they do.  `product` must
pass (tests/test_dp_graph_gpu.py runs it).  One rank.
"""
import os
import sys
import time

import torch
import torch.distributed as dist


def product(dev, G):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import ov3d_import
    ov3d_import.load()
    from ov3d_amd import dist as pdist
    params = [torch.nn.Parameter(torch.randn(n, device=dev)) for n in (1000, 3000, 257)]
    for p in params:
        p.grad = torch.ones_like(p)
    buckets = pdist.GradBuckets([params[:2], params[2:]], group=G)
    x = torch.ones(1 << 16, device=dev)
    eager = pdist.dedicated_stream(dev, "eager")
    cap = pdist.dedicated_stream(dev, "capture")
    eager.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(eager):
        for _ in range(3):
            dist.all_reduce(x)                 # SyncBN-like, WORLD group, on the eager stream
            buckets.launch(0)
            buckets.finish()                   # bucket_eager stream
    cap.wait_stream(eager)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(cap):               # no synchronize: the eager works are in flight
        g.capture_begin(capture_error_mode="thread_local")
        dist.all_reduce(x)
        buckets.launch(0)
        views = buckets.finish()
        t0 = time.time()
        while time.time() - t0 < 1.5:
            time.sleep(0.05)
        g.capture_end()
    torch.cuda.current_stream().wait_stream(cap)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    assert all(bool((views[id(p)] == 1).all()) for p in params)
    print("product: ok", flush=True)
    time.sleep(0.5)
    dist.destroy_process_group()


def main(mode):
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=os.environ.get("MASTER_PORT", "29531"),
                      TORCH_NCCL_CUDA_EVENT_CACHE="0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method="env://", world_size=1, rank=0, device_id=dev)
    G = dist.new_group([0], device_id=dev)
    if mode == "product":
        return product(dev, G)
    cap_group = dist.new_group([0], device_id=dev) if mode == "twin" else G
    x = torch.ones(1 << 20, device=dev)
    y = torch.ones(1 << 20, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    e = torch.cuda.Stream()
    e.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(e if mode == "estream" else s):
        for _ in range(4):
            w = dist.all_reduce(x, group=G, async_op=mode == "async")   # on G's watchdog list
            if w is not None:
                w.wait()
    s.wait_stream(e)
    with torch.cuda.stream(s):
        g.capture_begin(capture_error_mode="thread_local")
        dist.all_reduce(y, group=cap_group)    # cap_group's internal stream joins the capture
        # hold the capture open across several watchdog passes (~100 ms apart)
        t0 = time.time()
        while time.time() - t0 < 1.5:
            time.sleep(0.05)
        g.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print(f"{mode}: ok, y[0] = {y[0].item()}", flush=True)
    time.sleep(0.5)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])

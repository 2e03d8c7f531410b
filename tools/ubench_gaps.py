"""Launch-gap microbenchmark: an 800 MB int64 fill repeated on one stream, alone and with the
cross-stream event traffic the V2 lookahead puts between two replays (an event record after
each launch, a wait on a side-stream event before it, a small side-stream kernel per step)."""
import time
import torch

dev = torch.device("cuda:0")
x = torch.empty(100_000_000, dtype=torch.int64, device=dev)
y = torch.empty(1 << 20, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
side = torch.cuda.Stream(priority=0)
K = 200

def run(name, rec, wait, sidek, side_wait=True):
    evr = [torch.cuda.Event() for _ in range(3)]
    evd = [torch.cuda.Event() for _ in range(3)]
    for e in evd:
        e.record(side)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        if wait:
            s.wait_event(evd[i % 3])
        x.fill_(i)
        if rec:
            evr[i % 3].record(s)
        if sidek:
            with torch.cuda.stream(side):
                if rec and side_wait:
                    side.wait_event(evr[(i + 1) % 3])
                y.fill_(i)
                evd[(i + 2) % 3].record(side)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K
    print(f"{name:28s} {dt * 1e6:7.1f} us/launch", flush=True)

for rep in range(2):
    run("plain", False, False, False)
    run("record", True, False, False)
    run("wait", False, True, False)
    run("record+wait", True, True, False)
    run("record+wait+side kernel", True, True, True)
    run("side kernel only", False, False, True)
    run("side kernel, side waits", True, False, True)
    run("side kernel, main waits", True, True, True, side_wait=False)

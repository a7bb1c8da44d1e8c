"""How long does a fresh process's device allocation wait after another
process freed a large amount of HBM?  Child 1 fills and frees FILL GB; child 2
then times hipMalloc of sizes X1, X2, ... GB (each freed before the next).
Usage: python tools/alloc_wipe_probe.py FILL_GB X1 [X2 ...]
"""
import subprocess
import sys

fill = int(sys.argv[1])
sizes = [int(x) for x in sys.argv[2:]]
FILL = f"""
import torch, time
t0 = time.time()
xs = [torch.ones(1 << 30, dtype=torch.uint8, device='cuda') for _ in range({fill})]
torch.cuda.synchronize()
print('filled', len(xs), 'GB in', round(time.time() - t0, 2), 's', flush=True)
"""
PROBE = f"""
import torch, time
torch.cuda.init()
free, total = torch.cuda.mem_get_info()
print('free', round(free / 2**30, 1), 'of', round(total / 2**30, 1), 'GiB', flush=True)
for x in {sizes}:
    t0 = time.time()
    a = torch.empty(x << 30, dtype=torch.uint8, device='cuda')
    torch.cuda.synchronize()
    t1 = time.time()
    a.fill_(1)
    torch.cuda.synchronize()
    t2 = time.time()
    print('alloc', x, 'GiB', round((t1 - t0) * 1e3, 1), 'ms, first touch', round((t2 - t1) * 1e3, 1), 'ms', flush=True)
    del a
    torch.cuda.empty_cache()
"""
if fill:
    subprocess.run([sys.executable, "-c", FILL], check=True, timeout=120)
subprocess.run([sys.executable, "-c", PROBE], check=True, timeout=120)

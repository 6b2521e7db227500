"""Diagnostic: D2H rate into each of several page-locked host blocks (torch's caching
host allocator), to see whether some blocks are consistently slower (e.g. placed on
another NUMA node).  python tools/d2h_blocks.py [n_blocks] [MiB]"""
import sys
import torch

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 6
mib = int(sys.argv[2]) if len(sys.argv) > 2 else 64
n = mib << 20
dev = torch.empty(n, dtype=torch.uint8, device='cuda')
blocks = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(nb)]
st = torch.cuda.Stream(priority=-1)
for rep in range(3):
    rates = []
    for b in blocks:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            e0.record(st)
            b.copy_(dev, non_blocking=True)
            e1.record(st)
        st.synchronize()
        rates.append(n / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    print('rep %d GB/s per block: %s' % (rep, ' '.join('%.1f' % r for r in rates)), flush=True)

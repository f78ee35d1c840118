"""1-rank RCCL reduce_scatter_tensor: exactness over sizes / output offsets (tail handling)."""
import os

import torch
import torch.distributed as dist

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29734")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
big = torch.zeros(1 << 21, device="cuda")
for n in (66304, 65536, 66240, 1000, 4100, 131072 + 64, 7):
    for op in (dist.ReduceOp.AVG, dist.ReduceOp.SUM):
        for off in (0, 64, 66304):
            x = torch.randn(n, device="cuda")
            big.zero_()
            out = big[off:off + n]
            dist.reduce_scatter_tensor(out, x, op=op)
            torch.cuda.synchronize()
            d = (out - x).abs()
            bad = int((d > 0).sum())
            where = [] if bad == 0 else torch.nonzero(d > 0).flatten()[:6].tolist()
            print(f"n={n} op={op} off={off}: mismatches {bad} at {where}", flush=True)
dist.destroy_process_group()

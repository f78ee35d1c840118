"""Summarise a rocprofv3 kernel trace of the ZeRO-3 streamed-offload step: the last step's window
(between the last two adamw_commit kernels), busy time of the AdamW updates, of everything else, and
their overlap."""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        q = r.get("Queue_Id", "?") + "/" + r.get("Stream_Id", "?") + " #" + r.get("Correlation_Id", "?")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"] + " @" + q))
if len(sys.argv) > 2:
    print("columns:", list(r.keys()))
rows.sort()
commits = [r for r in rows if "adamw_commit" in r[2]]
print(f"kernels {len(rows)}  commits {len(commits)}")
t0, t1 = commits[-3][1], commits[-2][1]  # (the last commit is the end-of-training flush)
win = [r for r in rows if r[0] >= t0 and r[1] <= t1]
print(f"window {(t1 - t0) / 1e6:.2f} ms, {len(win)} kernels")


def union(iv):
    tot, cur = 0, None
    for s, e in sorted(iv):
        if cur is None or s > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    if cur:
        tot += cur[1] - cur[0]
    return tot


opt = [(s, e) for s, e, n in win if "adamw_kernel" in n]
oth = [(s, e) for s, e, n in win if "adamw_kernel" not in n]
uo, ur, ua = union(opt), union(oth), union(opt + oth)
print(f"adamw updates: {len(opt)} kernels, busy {uo / 1e6:.2f} ms (sum {sum(e - s for s, e in opt) / 1e6:.2f} ms)")
print(f"other kernels: busy {ur / 1e6:.2f} ms;  union {ua / 1e6:.2f} ms;  overlap {(uo + ur - ua) / 1e6:.2f} ms")
for s, e in opt[:6]:
    print(f"  update at +{(s - t0) / 1e6:8.2f} ms  dur {(e - s) / 1e6:.3f} ms")
# the first forward GEMM after the window start, the first backward marker
names = {}
for s, e, n in win:
    k = n.split("(")[0][:60]
    names[k] = names.get(k, 0) + (e - s)
for k, v in sorted(names.items(), key=lambda x: -x[1])[:15]:
    print(f"  {v / 1e6:9.2f} ms  {k}")

# the sequence around the update chain: 15 kernels before the first update, then every kernel until 40
# past it, with start offsets and durations
first = next(i for i, r in enumerate(win) if "adamw_kernel" in r[2])
print("sequence:")
for s, e, n in win[max(0, first - 10):first + 30]:
    print(f"  +{(s - t0) / 1e6:8.3f} ms  {(e - s) / 1e3:8.1f} us  {n.split('(')[0][:70]} {n.split('@')[-1]}")
print("first kernels of the window:")
for s, e, n in win[:12]:
    print(f"  +{(s - t0) / 1e6:8.3f} ms  {(e - s) / 1e3:8.1f} us  {n.split('(')[0][:70]} {n.split('@')[-1]}")

if len(sys.argv) > 3:  # HIP API calls longer than 1 ms inside the window
    api = []
    with open(sys.argv[3]) as f:
        for r in csv.DictReader(f):
            s_, e_ = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s_ >= t0 - 50_000_000 and s_ <= t1 and e_ - s_ > 1_000_000:
                api.append((s_, e_, r["Function"], r.get("Thread_Id", "?")))
    print("HIP API calls > 1 ms (window-relative):")
    for s_, e_, fn, th in sorted(api)[:40]:
        print(f"  +{(s_ - t0) / 1e6:8.3f} ms  {(e_ - s_) / 1e6:8.3f} ms  {fn}  thread {th}")

if len(sys.argv) > 3:  # host launch time of the kernels around the chain (correlation id -> API call start)
    launch = {}
    with open(sys.argv[3]) as f:
        for r in csv.DictReader(f):
            launch[r.get("Correlation_Id")] = (int(r["Start_Timestamp"]), r["Function"])
    print("device start vs host launch (window-relative ms):")
    sel = [r for r in win if "adamw" in r[2]][:4] + [r for r in win if "adamw" in r[2]][-3:]
    nxt = [r for r in rows if r[0] > t1][:8]
    for s_, e_, n in sel + nxt:
        cid = n.split("#")[-1].strip()
        h = launch.get(cid)
        hs = f"{(h[0] - t0) / 1e6:9.3f} ({h[1]})" if h else "?"
        print(f"  dev +{(s_ - t0) / 1e6:9.3f}  host {hs}  {n.split('(')[0][:50]}")


#!/usr/bin/env python3
"""Per-dispatch durations of the wg_verify_desc kernels in a rocprofv3
kernel trace of tools/verify_first_call.py: the first
call on each fresh stream against the calls after it.

usage: first_call_trace.py <rocprofv3 results .db> [note]   (prints one JSON object)

The tool's trials are the streams with exactly 6 verify dispatches (the
settling calls run on the default stream, hundreds of them); the first 8 such
streams in time are the 64-B batch, the next 8 the 1500-B batch."""
import json
import sqlite3
import statistics
import sys

ALG = {"64B": 1048576 * (64 + 16 + 1 + 2), "1500B": 1048576 * (1500 + 16 + 1 + 2)}


def main():
    db, note = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    c = sqlite3.connect(db)
    rows = c.execute("select stream_id, queue_id, start, end, name from kernels order by start").fetchall()
    streams, first_on_queue = {}, {}
    for sid, q, s, e, name in rows:
        first_on_queue.setdefault(q, s)  # the HW queue's first dispatch in the process
        if "verify" in name:
            streams.setdefault(sid, []).append((s, (e - s) / 1e3, name.split("(")[0], q))
    trials = sorted((v for v in streams.values() if len(v) == 6), key=lambda v: v[0][0])
    if len(trials) != 16:
        sys.exit(f"expected 16 six-call streams, found {len(trials)}")
    out = {"source": f"rocprofv3 --kernel-trace --stats -- python3 tools/verify_first_call.py ({db}); "
                     "kernel durations per dispatch; 8 fresh torch streams per size, 6 calls each",
           "algorithmic_bytes": dict(ALG, per_packet="len + 16 (descriptor) + 1 (verdict) + 2 (L4 result)")}
    for k, size in enumerate(("64B", "1500B")):
        tr = trials[8 * k: 8 * k + 8]
        first = [t[0][1] for t in tr]
        fresh = [first_on_queue[t[0][3]] == t[0][0] for t in tr]
        reused = [x for x, f in zip(first, fresh) if not f]
        later = [d for t in tr for (_, d, _, _) in t[2:]]
        fm, lm = statistics.median(first), statistics.median(later)
        out[size] = {"first_call_kernel": tr[0][0][2], "first_call_us": [round(x, 3) for x in first],
                     "first_call_us_median": round(fm, 3),
                     "first_call_frac_of_8TBps": round(ALG[size] / (fm * 1e-6) / 8e12, 4),
                     "hw_queue": [t[0][3] for t in tr],
                     "first_dispatch_on_its_hw_queue": fresh,
                     "first_call_us_median_queue_used_before": round(statistics.median(reused), 3) if reused else None,
                     "later_calls_us_median": round(lm, 3),
                     "later_frac_of_8TBps": round(ALG[size] / (lm * 1e-6) / 8e12, 4),
                     "kernels_per_stream": [[n for (_, _, n, _) in tr[0]]],
                     "calls_us_per_stream": [[round(d, 2) for (_, d, _, _) in t] for t in tr]}
    if note:
        out["note"] = note
    print(json.dumps(out))


if __name__ == "__main__":
    main()

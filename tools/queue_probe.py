#!/usr/bin/env python
"""Which streams share a hardware queue with the device-PNG decode stream?  Creates the streams
the batch pipeline creates, in its order, keeps the decode stream busy (torch.cuda._sleep ~100 ms)
and times a tiny op on each other stream: ~0 ms = its own queue, ~100 ms = queued behind the
sleep.  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from structured_light_for_3d_model_replication_amd import pipeline as PL  # noqa: E402

torch.cuda.init()
x = torch.zeros(1024, device="cuda")
streams = {"default": torch.cuda.current_stream(), "copy": torch.cuda.Stream(), "compute": torch.cuda.Stream(),
           "format": torch.cuda.Stream(), "decode": PL.png_decode_stream()}
out = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}
for rep in range(2):
    res = {}
    for name, st in streams.items():
        if name == "decode":
            continue
        torch.cuda.synchronize()
        with torch.cuda.stream(streams["decode"]):
            torch.cuda._sleep(250_000_000)               # ~100 ms at ~2.4 GHz
        time.sleep(0.005)
        t = time.perf_counter()
        with torch.cuda.stream(st):
            x.add_(1.0)
        st.synchronize()
        res[name] = round((time.perf_counter() - t) * 1e3, 2)
        torch.cuda.synchronize()
    out[f"rep{rep}_ms"] = res
t = time.perf_counter()
with torch.cuda.stream(streams["decode"]):
    torch.cuda._sleep(250_000_000)
streams["decode"].synchronize()
out["sleep_ms"] = round((time.perf_counter() - t) * 1e3, 2)
print(json.dumps(out))

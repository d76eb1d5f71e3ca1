"""Count host-synchronising HIP API calls in a ``rocprofv3 --hip-trace`` CSV.

VERDICT item: a pipeline step must not synchronise the host with the device.  Given the
``*_hip_api_trace.csv`` files of one run, prints per process the calls that block the host
until device work finishes (stream / device / event synchronize, blocking memcpy, queries
that are polled) and the total number of kernel-launch calls, so "syncs per step" can be read
off against the step count of the run.

    python tools/hip_sync_count.py gpurun_out/prof_pipe_r0 [--steps 200]
"""
import argparse
import csv
import json
import re
from collections import Counter
from pathlib import Path

SYNC = re.compile(r"^hip(StreamSynchronize|DeviceSynchronize|EventSynchronize|Memcpy|MemcpyDtoH|"
                  r"MemcpyHtoD|MemcpyWithStream|StreamWaitEvent|StreamQuery|EventQuery|Memset)$")
LAUNCH = re.compile(r"^hip(LaunchKernel|ExtLaunchKernel|ModuleLaunchKernel|GraphLaunch|"
                    r"ExtModuleLaunchKernel)$")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--steps", type=int, default=None)
    a = ap.parse_args()
    for d in a.dirs:
        files = sorted(Path(d).rglob("*hip_api_trace.csv"))
        for f in files:
            cnt, launches = Counter(), 0
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    fn = row.get("Function") or row.get("Operation") or ""
                    if SYNC.match(fn):
                        cnt[fn] += 1
                    if LAUNCH.match(fn):
                        launches += 1
            out = {"file": str(f), "launch_calls": launches, "host_sync_calls": dict(cnt)}
            if a.steps:
                # hipStreamWaitEvent orders streams on the device; hipEventQuery / hipStreamQuery
                # are non-blocking polls (the caching allocator's cross-stream frees)
                blocking = sum(v for k, v in cnt.items()
                               if k not in ("hipStreamWaitEvent", "hipMemset", "hipEventQuery",
                                            "hipStreamQuery"))
                out["blocking_per_step"] = round(blocking / a.steps, 3)
            print(json.dumps(out))


if __name__ == "__main__":
    main()

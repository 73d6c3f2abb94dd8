"""SHA-256 throughput of this host's cores, the way the multiproof transcript uses one: 4.9 MB hashed
on one thread, 30 times, each timed (hashlib: OpenSSL's SHA-NI path), then the same with a second
thread spinning beside it -- to tell the host core's clock (bimodal alone) from interference.
usage: sha_clock_probe.py"""
import hashlib
import os
import threading
import time

buf = os.urandom(4_915_200)


def run(tag, n=30):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        hashlib.sha256(buf).digest()
        ts.append((time.perf_counter() - t0) * 1e3)
        time.sleep(0.002)  # idle between hashes, as the bench's proofs are
    ts.sort()
    print(f"{tag}: min {ts[0]:.2f} p25 {ts[len(ts) // 4]:.2f} median {ts[len(ts) // 2]:.2f} "
          f"p75 {ts[3 * len(ts) // 4]:.2f} max {ts[-1]:.2f} ms  all {[round(x, 2) for x in sorted(ts)]}", flush=True)


run("alone")
stop = False


def spin():
    x = 0
    while not stop:
        x += 1


th = threading.Thread(target=spin)
th.start()
run("beside a spinning thread")
stop = True
th.join()
run("alone again")

"""What a resident RCCL receive costs the persistent decode step (VERDICT r5
item 7).

At N > 1 rank 0 posts the end-of-step gather (gpt2_decode_gather: grouped
ncclSend/ncclRecv on the comm stream, behind the step's logits copy) and the
next step's kernels start while the receive kernel waits for its peers' data.
RCCL 7.2 runs that receive as ncclDevKernel_Generic: one workgroup per channel
with 248-256 VGPRs and 37,664 B of LDS (the code object's metadata), so a CU
holding one cannot also hold a 12-wave chain workgroup, and the persistent
launches of the next step wait for it to exit.

One GPU cannot run two RCCL ranks, so the receive is tests/helpers/libocc.so's
recv_like_kernel: the same resources, launched behind an event on the decode
stream after every step (where the gather sits) and held for D us -- the time
the peers' data take to arrive after it is posted.  Steps are enqueued back
to back with no host sync, as bench.py's timed loop does, and the per-step
time is compared with the same loop without the receive.

The last cases run the library's own gather (gpt2_decode_gather: the send
copy, the compute -> comm hand-off, RCCL's grouped send/recv) on a 1-rank
communicator, logits and ids, every step.

usage: python tools/recv_coresidency.py [B ...]      (default: 8 64)
       (HPA_LIB=... picks the library, e.g. an A/B build)
"""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))
import pagedattn  # noqa: E402

LDS = 37664  # ncclDevKernel_Generic's group segment
CHUNK, CHUNKS = 100, 3


def main():
    Bs = [int(a) for a in sys.argv[1:]] or [8, 64]
    L = pagedattn.lib()
    occ = ctypes.CDLL(os.path.join(REPO, "tests", "helpers", "libocc.so"))
    occ.occ_recv_after.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.c_int,
                                   ctypes.c_void_p, ctypes.c_int]
    occ.occ_recv_after.restype = ctypes.c_int
    occ.occ_sync.restype = ctypes.c_int
    occ.occ_ring_record.argtypes = [ctypes.c_void_p, ctypes.c_int]
    cfgd = dict(pagedattn.GPT2_124M)
    ctx, start = cfgd["maxT"], cfgd["maxT"] - CHUNK - 8
    for B in Bs:
        m = pagedattn.Model(cfgd, seed=1337)
        m.decode_init(B, 16, ctx)
        m.reserve(ctx)
        m.fill_random(start, seed=77)
        m.set_graph(True)
        done = pagedattn.DeviceBuffer.from_array(np.zeros(1, np.int32))
        stream = L.hpa_get_stream()
        print(f"B={B}: layer form {m.layer_form()}", flush=True)

        def run(blocks, threads, us, mode=7, gather=-1):
            best, enq = [], []
            for _ in range(CHUNKS):
                m.set_positions(np.full(B, start, np.int32))
                pagedattn.check(L.hpa_device_synchronize(), "sync")
                t0 = time.perf_counter()
                for k in range(CHUNK):
                    m.step_async(None)
                    if mode & 64:  # host-deferred: post step k-1's receive once the host sees it done
                        assert occ.occ_ring_record(stream, k % 4) == 0
                        if k:
                            assert occ.occ_ring_wait((k - 1) % 4) == 0
                            rc = occ.occ_recv_after(stream, blocks, threads, int(us * 100), LDS, done.ptr, 4)
                            assert rc == 0, rc
                    elif gather >= 0:
                        m.gather(gather)
                    elif mode:
                        rc = occ.occ_recv_after(stream, blocks, threads, int(us * 100), LDS, done.ptr, mode)
                        assert rc == 0, rc
                enq.append((time.perf_counter() - t0) * 1e3 / CHUNK)
                pagedattn.check(L.hpa_device_synchronize(), "sync")
                best.append((time.perf_counter() - t0) * 1e3 / CHUNK)
                m.status()  # a timed-out in-launch wait raises
            return min(best), min(enq)

        for _ in range(3):  # warm the graph, the clocks
            run(0, 0, 0, 0)
        base, e0 = run(0, 0, 0, 0)
        print(f"  alone: {base:.4f} ms/step (host enqueue {e0 * 1e3:.1f} us/step)", flush=True)
        cases = [(1, 64, 0, "event recorded on the decode stream only"),
                 (3, 64, 0, "event recorded + helper stream waits on it, no kernel"),
                 (4, 64, 0, "64 x 512 recv-like, held 0 us, no dependency on the step"),
                 (6, 64, 0, "helper stream waits on a stale event, 64 x 512 held 0 us")]
        cases += [(3 | (k << 3), 64, 0, f"event + wait, no kernel; event flags: {f}")
                  for k, f in ((1, "DisableSystemFence"), (2, "ReleaseToDevice"))]
        cases += [(35, 64, 0, "stream write-value + wait-value, no kernel"),
                  (39, 64, 0, "write-value + wait-value + 64 x 512 held 0 us"),
                  (64, 64, 0, "host-deferred: host waits step k-1, posts 64 x 512 held 0 us"),
                  (64, 64, 100, "host-deferred: host waits step k-1, posts 64 x 512 held 100 us"),
                  (64, 8, 100, "host-deferred: host waits step k-1, posts 8 x 512 held 100 us")]
        cases += [(7, b, us, f"gather pattern: {b:3d} x 512 recv-like held {us:3d} us")
                  for b in (8, 32, 64) for us in (0, 50, 100, 200)]
        for mode, b, us, what in cases:
            t, e = run(b, 512, us, mode)
            print(f"  {what:64s} {t:.4f} ms/step (+{(t - base) * 1e3:6.1f} us; enqueue {e * 1e3:.1f} us)",
                  flush=True)
        assert occ.occ_sync() == 0
        n = L.hpa_comm_id_bytes()
        uid = ctypes.create_string_buffer(n)
        pagedattn.check(L.hpa_comm_unique_id(uid, n), "unique id")
        pagedattn.check(L.hpa_comm_init(1, 0, uid), "comm init")
        m.shard([B], root=0)
        for what in (0, 1):
            t, e = run(0, 0, 0, 0, gather=what)
            print(f"  {'library gather, 1-rank RCCL: ' + ('logits' if what == 0 else 'ids'):64s} {t:.4f} ms/step "
                  f"(+{(t - base) * 1e3:6.1f} us; enqueue {e * 1e3:.1f} us)", flush=True)
        m.close()
        pagedattn.check(L.hpa_comm_destroy(), "comm destroy")


if __name__ == "__main__":
    main()

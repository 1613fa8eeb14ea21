"""Deadline on the device synchronisation of a sharded run (the first multi-GPU run must fail
diagnosably, not hang).

A lost or stalled peer does not fail on the host: RCCL's send / recv wait inside their kernels, so the host's next
device synchronise would block forever.  `guarded_sync` marks the stream (hdd_block_step_mark), then synchronises
with a watchdog thread beside it: if the deadline passes first, the watchdog asks the library which stage of the
rank's last sharded step has not completed (hdd_block_step_query: halo pack, halo exchange, ghost-adjacent element
pass, tile assembly and join), prints the rank, the stage and the halo peers to stderr and ends the process with a
non-zero status (os._exit: no re-exec, no retry, no Python teardown that could block on the device again).

Coverage: the stage report needs device-side stage events, which the RCCL and in-process device transports record
(the exchange runs on the device).  The host transport (hdd_comm_create_host: gloo, MPI, a mailbox -- bench.py's
`--backend gloo` rehearsal) exchanges synchronously inside the step call, before this guard is armed: a stalled peer
blocks there and is bounded only by the transport's own timeout (the gloo process group's, >= 120 s in bench.py),
and no stage is named.
"""
import os
import sys
import threading

EXIT_STATUS = 3


def report(shard, rank, what, deadline, stage_name):
    try:
        peers = [int(p) for p in shard.halo_lists()[0]]
    except Exception:   # noqa: BLE001 -- best effort inside the failure path
        peers = "?"
    return ("[hdd watchdog] rank %d: %s did not complete within %.0f s -- stage '%s' of the sharded step has not "
            "completed (halo peers %s)" % (rank, what, deadline, stage_name, peers))


def guarded_sync(torch, shard, rank, what, deadline, on_timeout=None, stream=None):
    """torch.cuda.synchronize() under a deadline (seconds).  On expiry: print the stage report to stderr, call
    on_timeout() if given (tests: open an injected gate so the device drains), then os._exit(EXIT_STATUS)."""
    shard.step_mark(stream)
    done = threading.Event()

    def dog():
        if done.wait(deadline):
            return
        try:
            stage = shard.step_query()[1]
        except Exception as e:   # noqa: BLE001
            stage = "unknown (%s)" % e
        sys.stderr.write(report(shard, rank, what, deadline, stage) + "\n")
        sys.stderr.flush()
        sys.stdout.flush()
        if on_timeout is not None:
            try:
                on_timeout()
            except Exception:   # noqa: BLE001
                pass
        os._exit(EXIT_STATUS)

    t = threading.Thread(target=dog, name="hdd-watchdog", daemon=True)
    t.start()
    torch.cuda.synchronize()
    done.set()
    t.join()

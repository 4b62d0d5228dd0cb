"""A consumer process for the CUDA-IPC tests (torch.multiprocessing's CUDA tensor sharing, what
the reference's PipeServerEndpoint.broadcast does with a result): it rebuilds what it is sent, reads
it, releases it and exits, so the producer's IPC limbo drains before the producer ends."""

from __future__ import annotations


def consume(conn) -> None:
    from multiprocessing.reduction import ForkingPickler

    import torch
    import torch.multiprocessing  # noqa: F401  (registers the tensor rebuilders)

    obj = ForkingPickler.loads(conn.recv_bytes())
    tensors = list(obj.values()) if isinstance(obj, dict) else [obj]
    total = sum(float(t.double().sum().item()) for t in tensors)
    del obj, tensors
    torch.cuda.synchronize()
    conn.send(total)
    conn.close()


def hand_over(payload: bytes) -> float:
    """Send ``payload`` (ForkingPickler.dumps of CUDA tensors) to a fresh consumer process and wait
    until it has released them; returns the sum it read."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    parent, child = ctx.Pipe()
    p = ctx.Process(target=consume, args=(child,))
    p.start()
    parent.send_bytes(payload)
    total = parent.recv()
    p.join(timeout=120)
    assert p.exitcode == 0, p.exitcode
    return total

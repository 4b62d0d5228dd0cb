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


def produce(conn, shapes: dict, seeds: list) -> None:
    """A worker process on the same GPU: makes one update per seed on cuda:0 and sends it through
    torch.multiprocessing (CUDA IPC, what the reference's pipes do with CUDA tensors), then keeps
    the tensors alive until the receiver says it is done."""
    import torch
    import torch.multiprocessing  # noqa: F401  (registers the tensor reducers)
    from multiprocessing.reduction import ForkingPickler

    dev = torch.device("cuda", 0)
    kept = []
    for s in seeds:
        g = torch.Generator().manual_seed(s)
        upd = {name: torch.randn(sh, generator=g).to(dev) for name, sh in shapes.items()}
        kept.append(upd)
        conn.send_bytes(bytes(ForkingPickler.dumps(upd)))
    torch.cuda.synchronize()
    conn.recv()  # the receiver is done with them
    del kept
    conn.close()

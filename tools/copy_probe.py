"""Which part of a run leaves async memory copies undelivered at exit (rocprofv3
--memory-copy-trace prints "timed out ... waiting for N completion callbacks")?
    python tools/copy_probe.py {torch|engine|bench-like}
torch: a torch H2D/D2H round trip only; engine: a small snapshot, an engine, pinned and
pageable host batches, everything closed explicitly before exit."""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])


def main(kind):
    a = torch.ones(1 << 20, device="cuda")
    b = a.cpu()
    torch.cuda.synchronize()
    if kind == "torch":
        return
    from keto_amd import check, synth
    from keto_amd.snapshot import Snapshot
    w = synth.rbac(users=20000, groups=2000, docs=4000, tuples=120000, checks=20000, seed=9)
    snap = Snapshot.from_columns(w.namespaces, w.columns)
    r, t = w.resolve(snap)
    eng = check.Engine(snap)
    pr, pt = check.pinned(r), check.pinned(t)
    out = check.PinnedBuffer((len(r) + 63) // 64, np.uint64)
    for _ in range(3):
        eng.check_ids_raw(pr.array.ctypes.data, pt.array.ctypes.data, len(r), out.array.ctypes.data)
        eng.check_ids(r, t)
    q = eng.upload(r, t)
    q.run()
    q.download()
    del q
    for x in (pr, pt, out):
        x.close()
    eng.close()
    torch.cuda.synchronize()
    print("engine probe done", b.sum().item())


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "engine")

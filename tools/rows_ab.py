"""Same-process A/B of the masked workloads' rows-first representation modifier (models.encode_rows runs the
position-wise modifier on the selected rows only) against the modifier on every position followed by the row
selection: bench.bench_bert4rec alternated with the modifiers' forward_rows hidden.
Usage: python tools/rows_ab.py [bert4rec|kebert4rec] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402
import bench  # noqa: E402

workload = sys.argv[1] if len(sys.argv) > 1 else "bert4rec"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
items = 27000 if workload == "bert4rec" else 13000
sys.argv = ["bench.py", "--workload", workload, "--items", str(items), "--steps", "20", "--warmup", "5",
            "--cpu-baseline", "0", "--legs", "none"]
args = bench.parse()
asme = __graft_entry__.load_package()
dev = torch.device("cuda", 0)
classes = [asme.layers.FFNSequenceRepresentationModifierComponent,
           asme.layers.PostFusionContextSequenceRepresentationModifierComponent,
           asme.layers.IdentitySequenceRepresentationModifierLayer,
           asme.layers.PostFusionIdentitySequenceRepresentationModifierLayer]
saved = {c: c.forward_rows for c in classes}
for rep in range(reps):
    for rows_first in (True, False):
        for c in classes:
            if rows_first:
                c.forward_rows = saved[c]
            elif "forward_rows" in c.__dict__:
                del c.forward_rows
        r = bench.bench_bert4rec(args, asme, dev, 1, 0, workload, items)
        print(f"{workload} rows_first={rows_first}: {r['value']:.1f} seq/s {r['ms_per_step']:.3f} ms/step", flush=True)

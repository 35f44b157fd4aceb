"""HBM traffic per launch of the config-2 IL backward (the launch bench.py's roofline times) from
two rocprofv3 PMC passes over the SAME bench command (tools/measure.sh pmc): FETCH_SIZE and
WRITE_SIZE, separate passes (MI355X_MICROARCH.md: one counter group per pass), FETCH_SIZE x2
(gfx950 reports half of wide coalesced reads), WRITE_SIZE as is; KB per dispatch, averaged
over every dispatch of the kernel in the run (the timed steps and the roofline launches are the
same launch, rs_il_bwd_push_saved_xt).

    python tools/il_traffic.py <dir with pmc_FETCH_SIZE/ pmc_WRITE_SIZE/> <per-GPU batch> out.json
"""
import csv
import glob
import json
import sys

KERNEL = {True: "bwd4_kernel", False: "wbwd_kernel"}


def mean_counter(root, counter, kname):
    vals = []
    for f in glob.glob(f"{root}/pmc_{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and kname in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kname} under {root}")
    return sum(vals) / len(vals), len(vals)


def main(root, batch, out):
    batch = int(batch)
    kname = KERNEL[batch > 1536]
    fe, nf = mean_counter(root, "FETCH_SIZE", kname)
    wr, nw = mean_counter(root, "WRITE_SIZE", kname)
    hbm = (2 * fe + wr) * 1024
    # algorithmic bytes per launch: x0, xsave, the attention save, dy,
    # the head's dx0 share, rows in; pushed rows + flags, per-block partials, dW1 rows out
    res = {"kernel": f"rs_il::{kname}", "launch": "rs_il_bwd_push_saved_xt", "per_gpu_batch": batch,
           "hbm_bytes_per_launch": int(round(hbm)), "fetch_size_kb": fe, "write_size_kb": wr,
           "dispatches": [nf, nw],
           "correction": "FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads; "
                         "MI355X_MICROARCH.md HBM), WRITE_SIZE as is; both KB per dispatch",
           "source": f"rocprofv3 --kernel-trace --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) "
                     f"over bench.py --global-batch {batch} (tools/measure.sh pmc)"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:4])

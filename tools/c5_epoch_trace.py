"""C5 epoch loop from a rocprofv3 --kernel-trace CSV of tools/c5bench.py: per epoch launch the
producer (rng_kernel on its stream) and the walked resolve beside the next one, for the last call.
    python tools/c5_epoch_trace.py gpurun_out/<dir>/kt_kernel_trace.csv [epochs=33]"""
import csv
import sys


def main(path, ne=33):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "rng_kernel" in r["Kernel_Name"]]
    sub = rows[idx[-ne]:]
    t0 = int(sub[0]["Start_Timestamp"])

    def span(r):
        return (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3

    P = [span(r) for r in sub if "rng_kernel" in r["Kernel_Name"]]
    R = [span(r) for r in sub if "resolve" in r["Kernel_Name"]]
    print("producer mean %.1f us, resolve mean %.1f us, %d / %d launches" %
          (sum(e - s for s, e in P) / len(P), sum(e - s for s, e in R) / len(R), len(P), len(R)))
    for i in range(min(4, len(P))):
        print("  P%d %8.1f-%8.1f   R%d %8.1f-%8.1f" % (i, P[i][0], P[i][1], i, R[i][0], R[i][1]))
    print("  last P %.1f-%.1f  R %.1f-%.1f" % (P[-1] + R[-1]))
    for r in sub[-6:]:
        s, e = span(r)
        print("  %-40s %9.1f %9.1f" % (r["Kernel_Name"][:40], s, e))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 33)

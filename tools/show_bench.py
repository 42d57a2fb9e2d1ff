"""One summary line from a bench.py log: tools/show_bench.py <log> <label>.

Reads the last JSON line bench.py printed (rank 0) and prints the step time, the path kernel's
HIP-event time, the rate and, when present, the parity figures of the timed image."""
import json
import sys


def main():
    path, label = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    lines = [l for l in open(path) if l.startswith("{")]
    if not lines:
        print(f"{label}: no bench line in {path}")
        return 1
    d = json.loads(lines[-1])
    rf = d.get("roofline", {})
    par = d.get("parity") or {}
    extra = f", rmse {par['rmse']:.2e}, rays x{par['ray_ratio']:.6f}" if "rmse" in par else ""
    print(f"{label:>20}: {d['ms_per_step']:.3f} ms/step, kernel {rf.get('kernel_ms')} ms, "
          f"{d['value']:.0f} {d['unit']}, frac {rf.get('frac')}{extra} "
          f"[vgprs {rf.get('vgprs')}, lds {rf.get('lds_bytes')}, treelet {rf.get('tree_nodes')}, wg {rf.get('wg')}]")
    return 0


if __name__ == "__main__":
    sys.exit(main())

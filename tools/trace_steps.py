"""Per-step timeline of a rocprofv3 kernel trace: the dominant kernel's
launches (matched by a name substring) and, between consecutive ones, every
other kernel that ran, with its queue and its start/end relative to the
dominant launch it follows.  Prints a summary over the last `--last` steps.

  python tools/trace_steps.py TRACE.csv SUBSTR [--last 20] [--show 3]"""
import argparse
import csv
import statistics


def short(name):
    return name.split("(")[0].replace("void ", "")[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("substr")
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--show", type=int, default=2)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if r["Kind"] == "KERNEL_DISPATCH"]
    ks = sorted(({"name": short(r["Kernel_Name"]), "q": r["Queue_Id"], "s": int(r["Start_Timestamp"]),
                  "e": int(r["End_Timestamp"])} for r in rows), key=lambda k: k["s"])
    dom = [k for k in ks if a.substr in k["name"]]
    dom = dom[-(a.last + 1):]
    gaps, durs = [], []
    for i in range(len(dom) - 1):
        d0, d1 = dom[i], dom[i + 1]
        gaps.append((d1["s"] - d0["e"]) / 1e3)
        durs.append((d0["e"] - d0["s"]) / 1e3)
        if i >= len(dom) - 1 - a.show:
            print(f"--- {d0['name']} q{d0['q']} {durs[-1]:.1f} us, next starts {gaps[-1]:.1f} us after it ends")
            for k in ks:
                if k is d0 or k["e"] < d0["s"] or k["s"] > d1["s"]:
                    continue
                if a.substr in k["name"]:
                    continue
                print(f"    {k['name']:48s} q{k['q']} start {(k['s'] - d0['s']) / 1e3:8.1f}  end "
                      f"{(k['e'] - d0['s']) / 1e3:8.1f}  dur {(k['e'] - k['s']) / 1e3:7.1f} us")
    print(f"dominant: median {statistics.median(durs):.1f} us, gap to next median {statistics.median(gaps):.1f} us, "
          f"period median {statistics.median([g + d for g, d in zip(gaps, durs)]):.1f} us over {len(durs)} steps")


if __name__ == "__main__":
    main()

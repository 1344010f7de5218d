"""Extract the reference's PUBLISHED hep-th results into tests/golden/hep_th_published.json.

Run in the build container only (it reads /root/reference, which the GPU box does not have):
    python tests/golden/make_goldens.py
Sources (all data files that ship in the reference repo):
  data/quality/hep.degree.raw:8-12   TREEFAQS digest of the hep-th elimination tree
  data/quality/hep.degree.raw:13-..  partition_tree -f -g output for k = 2..32 (one run)
  data/quality/hep.cost:2-32         ECV(down) column "sheep-degree" for k = 2..32
  data/hep-th.dat.ini                vertices / edges header
The published log was produced by dist-partition.sh -w 2 on hep-th (scripts/part-worker.sh:24
runs partition_tree once with all k), so kids order persists across k (see oracle).
"""
import json
import os
import re

REF = "/root/reference/data"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hep_th_published.json")


def main():
    raw = open(os.path.join(REF, "quality/hep.degree.raw")).read()
    facts = dict((k, int(v)) for k, v in re.findall(r"(\w+):(\d+)", raw.split("Partitioning")[0])
                 if k in ("width", "roots", "vheight", "eheight", "verts", "edges", "halo",
                          "core", "fill"))
    blocks = raw.split("Partitioning took:")[1:]
    parts = []
    for b in blocks:
        g = lambda pat: re.search(pat, b)
        m = g(r"Actually created (\d+) partitions")
        s = g(r"First two partition sizes: (\d+) and (\d+)")
        rec = {"created": int(m.group(1)), "size0": int(s.group(1)), "size1": int(s.group(2))}
        for key, label in (("edges_cut", "edges cut"), ("vcom_vol", "Vcom. vol"),
                           ("ecv_hash", r"ECV\(hash\)"), ("ecv_down", r"ECV\(down\)"),
                           ("ecv_up", r"ECV\(up\)\s*")):
            mm = g(label + r": (\d+) \(([0-9.]+)%\)")
            rec[key] = int(mm.group(1))
            rec[key + "_pct"] = mm.group(2)
        parts.append(rec)
    cost = {}
    for line in open(os.path.join(REF, "quality/hep.cost")):
        f = line.split()
        if f and f[0].isdigit():
            cost[int(f[0])] = int(f[1])
    for i, rec in enumerate(parts):
        rec["k"] = i + 2
        assert cost[rec["k"]] == rec["ecv_down"], rec
    ini = dict(l.strip().split("=", 1) for l in open(os.path.join(REF, "hep-th.dat.ini"))
               if "=" in l)
    json.dump({"source": "arpang/sheep data/quality/hep.degree.raw, hep.cost, hep-th.dat.ini",
               "ini": {"vertices": int(ini["vertices"]), "edges": int(ini["edges"])},
               "treefaqs": facts, "partitions": parts}, open(OUT, "w"), indent=1)
    print("wrote", OUT, len(parts), "partition records")


if __name__ == "__main__":
    main()

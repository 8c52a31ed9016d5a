"""Fold an A/B evidence directory under profiles/ into one file.

    python tools/pack_profiles.py profiles/r03/c5ab [...]

Every file under the directory becomes one line of <dir>/ab_lines.jsonl:
{"file": <path relative to the directory>, "json": <parsed .json>} or
{"file": ..., "jsonl": [<parsed lines>]} or {"file": ..., "text": <the file's
text>}; the files are then removed (the history keeps them).  DESIGN.md cites
such directories as a whole; one line per former file keeps every number
while the tree stops growing by a file per A/B leg."""
import json
import os
import sys


def fold(d):
    out = os.path.join(d, "ab_lines.jsonl")
    recs, paths = [], []
    for root, _, files in os.walk(d):
        for f in sorted(files):
            p = os.path.join(root, f)
            if os.path.abspath(p) == os.path.abspath(out):
                continue
            rel = os.path.relpath(p, d)
            with open(p, "rb") as fh:
                raw = fh.read()
            try:
                txt = raw.decode()
            except UnicodeDecodeError:
                print("skip binary", p)
                continue
            rec = {"file": rel}
            try:
                if f.endswith(".json"):
                    rec["json"] = json.loads(txt)
                elif f.endswith(".jsonl"):
                    rec["jsonl"] = [json.loads(x) for x in txt.splitlines() if x.strip()]
                else:
                    rec["text"] = txt
            except ValueError:
                rec["text"] = txt
            recs.append(rec)
            paths.append(p)
    recs.sort(key=lambda r: r["file"])
    mode = "a" if os.path.exists(out) else "w"
    with open(out, mode) as fh:
        for r in recs:
            fh.write(json.dumps(r, separators=(",", ":")) + "\n")
    for p in paths:
        os.remove(p)
    for root, dirs, _ in os.walk(d, topdown=False):
        for x in dirs:
            q = os.path.join(root, x)
            if not os.listdir(q):
                os.rmdir(q)
    print(d, len(paths), "files ->", out)


if __name__ == "__main__":
    for d in sys.argv[1:]:
        fold(d)

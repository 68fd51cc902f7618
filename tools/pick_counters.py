"""Pick the counters of a wanted list that `rocprofv3 -L` reports on this box.

    python tools/pick_counters.py LIST_FILE NAME [NAME ...]  -> space-separated names

The wanted list must already respect the per-pass block limits (MI355X:
8 SQ, 4 TCC, 2 GRBM); unknown names are dropped, never substituted.
"""
import re
import sys


def main():
    text = open(sys.argv[1], errors="replace").read()
    have = set(re.findall(r"\b([A-Z][A-Z0-9_]+)\b", text))
    print(" ".join(n for n in sys.argv[2:] if n in have))


if __name__ == "__main__":
    main()

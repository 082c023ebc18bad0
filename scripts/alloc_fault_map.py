"""Map a GPU fault address to the native allocator's live blocks (replay of a PD_ALLOC_TRACE file).

usage: python scripts/alloc_fault_map.py TRACE_FILE FAULT_ADDR_HEX [LOG_FILE]
(with LOG_FILE, the address is taken from the HIP 'Memory access fault ... on address 0x...' line)."""
import bisect
import re
import sys


def main():
    path = sys.argv[1]
    addr = None
    if len(sys.argv) > 2 and not sys.argv[2].startswith("0x") and len(sys.argv) == 3:
        sys.argv.append(sys.argv[2])
    if len(sys.argv) > 3:
        m = re.search(r"address (0x[0-9a-fA-F]+)", open(sys.argv[3], errors="replace").read())
        addr = int(m.group(1), 16) if m else None
    if addr is None:
        addr = int(sys.argv[2], 16)
    live, order = {}, 0
    for ln in open(path):
        f = ln.split()
        if not f:
            continue
        if f[0] == "A" and len(f) >= 3 and f[1] != "(nil)":
            order += 1
            live[int(f[1], 16)] = (int(f[2]), order)
        elif f[0] == "F" and len(f) >= 2:
            live.pop(int(f[1], 16), None)
    starts = sorted(live)
    i = bisect.bisect_right(starts, addr) - 1
    print(f"fault address {addr:#x}; {len(live)} live blocks at the fault")
    for j in range(max(0, i - 3), min(len(starts), i + 4)):
        s = starts[j]
        size, o = live[s]
        rel = addr - s
        tag = "CONTAINS" if 0 <= rel < size else (f"+{rel - size:#x} past end" if rel >= size else f"{-rel:#x} before")
        print(f"  block {s:#x} size {size:>12} (alloc #{o}): {tag}")


if __name__ == "__main__":
    main()

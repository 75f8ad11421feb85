"""Turn rocprofv3 kernel_stats / counter CSVs into a committed markdown summary."""
import csv
import sys


def kernel_stats(path, top=15):
    rows = list(csv.DictReader(open(path)))
    out = ["| kernel | calls | avg us | total % |", "|---|---|---|---|"]
    for r in rows[:top]:
        name = r["Name"].replace("|", "/")
        if len(name) > 90:
            name = name[:87] + "..."
        out.append(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    return "\n".join(out)


if __name__ == "__main__":
    print(kernel_stats(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 15))

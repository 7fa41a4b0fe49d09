"""Per-proof kernel totals from a rocprofv3 kernel_stats.csv of a bench run:
    python tools/kstats.py run_kernel_stats.csv
Divides by the number of k_quotient_ launches (one per proof); one-time setup
kernels (SRS, folded table, circuit synthesis, key preparation) are listed
separately."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
proofs = sum(int(r["Calls"]) for r in rows if r["Name"].startswith(("pnp::k_quotient_", "pnp::k_quotient29_")))
setup = ("k_srs_", "k_table_", "k_synth", "k_coset_consts", "k_powers_table", "k_to_blocks", "k_fermat_inv")
tot = 0.0
print(f"{proofs} proofs")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    name = r["Name"].split("(")[0].replace("pnp::", "")
    ms = float(r["TotalDurationNs"]) / 1e6
    if any(s in name for s in setup):
        print(f"  [setup] {name:40s} {ms:9.2f} ms total")
        continue
    tot += ms / proofs
    if ms / proofs > 0.1:
        print(f"  {name:48s} {ms / proofs:8.2f} ms/proof  {int(r['Calls']) / proofs:6.1f} calls  {float(r['AverageNs']) / 1e3:9.1f} us avg")
print(f"kernel time per proof (excl. setup): {tot:.2f} ms")

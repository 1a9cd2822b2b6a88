"""Per-round, per-client table of a multi-round virtual-client bench record
(``bench.py --virtual-clients N --rounds R``: the ``per_round`` field of its JSON line).

    python scripts/fed_rounds_report.py gpurun_out/r6fed/fedavg_8x3_default.json.log [title]
"""
import json
import sys


def main(path, title=None):
    rec = None
    with open(path) as f:
        for line in f:
            if line.startswith("{"):
                rec = json.loads(line)
    if rec is None or "per_round" not in rec:
        raise SystemExit(f"{path}: no multi-round bench record")
    out = []
    out.append(title or f"{rec['quality_virtual_clients']} virtual clients x {rec['fedavg_rounds']} FedAvg rounds")
    out.append(f"source: {path}")
    out.append(f"protocol: {rec['quality_file_rows']:,}-row synthetic file, 10 % per client (seed 42 + k), "
               f"{rec['train_rows_per_client']:,} train / {rec['eval_rows_per_client']:,} test rows per client, "
               f"{rec['local_epochs']} local epochs per round (Adam lr {rec['quality_lr']}, fresh each round), "
               f"unweighted FedAvg; quality wall {rec['quality_wall_s']} s on one MI355X")
    out.append(f"throughput window of the same run: {rec['ms_per_step']} ms/step ({rec['value']} batches/s)")
    out.append("")
    hdr = (f"{'round':>5} {'client':>6} | {'local acc %':>11} {'local F1':>9} {'local [[TN,FP],[FN,TP]]':>28} | "
           f"{'agg acc %':>9} {'agg F1':>8} {'agg [[TN,FP],[FN,TP]]':>26} | {'rel L2 to agg':>13}")
    out.append(hdr)
    out.append("-" * len(hdr))
    for r in rec["per_round"]:
        for c in r["clients"]:
            out.append(f"{r['round']:>5} {c['client']:>6} | {c['local_accuracy_pct']:>11.3f} {c['local_f1']:>9.5f} "
                       f"{str(c['local_confusion']):>28} | {c['aggregated_accuracy_pct']:>9.3f} "
                       f"{c['aggregated_f1']:>8.5f} {str(c['aggregated_confusion']):>26} | "
                       f"{c['rel_l2_local_to_aggregate']:>13.4e}")
        out.append(f"{r['round']:>5} {'pooled':>6} | {r['local_accuracy_pct']:>11.3f} {r['local_f1']:>9.5f} "
                   f"{str(r['local_confusion']):>28} | {r['aggregated_accuracy_pct']:>9.3f} {r['aggregated_f1']:>8.5f} "
                   f"{str(r['aggregated_confusion']):>26} | worst client {r['min_client_aggregated_accuracy_pct']:.3f} % "
                   f"/ F1 {r['min_client_aggregated_f1']:.5f}")
        out.append("")
    bar = [(r["round"], r["aggregated_accuracy_pct"] >= 99.87 and r["aggregated_f1"] >= 0.998,
            r["min_client_aggregated_accuracy_pct"] >= 99.87 and r["min_client_aggregated_f1"] >= 0.998)
           for r in rec["per_round"]]
    out.append("reference bar (>= 99.87 % accuracy and >= 0.998 F1 after aggregation): "
               + "; ".join(f"round {k}: pooled {'met' if p else 'NOT met'}, every client {'met' if w else 'NOT met'}"
                           for k, p, w in bar))
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)

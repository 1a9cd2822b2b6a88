"""Does one FedAvg round lift each client?  The reference's 2-client round on a data profile where
the 3-epoch local models are NOT saturated (the reference: 99.09 / 99.05 % local -> 99.93 / 99.87 %
aggregated, client{1,2}_local_metrics.csv:2 vs client{1,2}_aggregated_metrics.csv:2).

    python scripts/fedavg_lift.py [lookalike fractions] [file seeds] [rows]     e.g.  0.03,0.06,0.1 0,1

Per (look-alike fraction, file seed): a 225,745-row synthetic file with that fraction of BENIGN rows
turned into flood-shaped HTTP flows (data/synthetic.py ``lookalike``, the "calibrated" profile's
knob), then fed/runner.py ``run_virtual_clients``: client k samples its 10 % with seed 42 + k, both
start from the same init, 3 local epochs each (bs32, Adam lr 2e-5), unweighted FedAvg (the fedavg_
sum + scale_cast), each client's test split evaluated on its local model and on the aggregate.
Prints one line per client and a JSON summary line (profiles/r5_fedavg_lift.txt)."""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd import config  # noqa: E402
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.data import generate_cicids2017  # noqa: E402,E501
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.fed import runner  # noqa: E402


def main():
    fracs = [float(a) for a in (sys.argv[1] if len(sys.argv) > 1 else "0.06").split(",")]
    seeds = [int(s) for s in (sys.argv[2] if len(sys.argv) > 2 else "0,1").split(",")]
    rows = int(sys.argv[3]) if len(sys.argv) > 3 else 225_745
    out = []
    for frac in fracs:
        for seed in seeds:
            t0 = time.perf_counter()
            frame = generate_cicids2017(rows, seed=seed, lookalike=frac)
            fc = config.FedConfig(synthetic_rows=rows, batch_size=32, eval_batch_size=16, epochs=3, rounds=1,
                                  max_len=128, impl="hip", out_dir=tempfile.mkdtemp(prefix="fedlift_"), plots=False,
                                  resume=False, save_checkpoints=False, heartbeat_s=0.0, verbose=False)
            client = runner.FederatedClient(fc, frame=frame)
            client.setup()
            res = runner.run_virtual_clients(client, 2)
            for c in res["clients"]:
                lo, ag = c["local_test"], c["aggregated_test"]
                rec = {"lookalike": frac, "file_seed": seed, "client": c["client"],
                       "local_acc": round(lo["accuracy"], 3), "local_f1": round(lo["f1"], 5),
                       "local_cm": lo["confusion_matrix"], "agg_acc": round(ag["accuracy"], 3),
                       "agg_f1": round(ag["f1"], 5), "agg_cm": ag["confusion_matrix"],
                       "lift_pct": round(ag["accuracy"] - lo["accuracy"], 3),
                       "rel_l2_local_to_agg": round(c["rel_l2_local_to_aggregate"], 5),
                       "epoch_losses": [round(x, 5) for x in c["train"]["epoch_losses"]]}
                out.append(rec)
                print(f"lookalike {frac:.3f} file {seed} client {c['client']}: local {rec['local_acc']:7.3f} % "
                      f"F1 {rec['local_f1']:.5f} cm {rec['local_cm']} -> aggregated {rec['agg_acc']:7.3f} % "
                      f"F1 {rec['agg_f1']:.5f} cm {rec['agg_cm']} (lift {rec['lift_pct']:+.3f}; "
                      f"|local - agg| / |local| {rec['rel_l2_local_to_agg']:.4f})", flush=True)
            print(f"  ({time.perf_counter() - t0:.1f} s)", flush=True)
            del client
    lifts = [r["lift_pct"] for r in out]
    print(json.dumps({"runs": out, "mean_lift_pct": round(sum(lifts) / max(len(lifts), 1), 3),
                      "clients_lifted": sum(x > 0 for x in lifts), "clients": len(lifts)}))


if __name__ == "__main__":
    main()

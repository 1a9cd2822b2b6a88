"""Command-line entry points (``python -m detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd <cmd>``).

  client   run federated client(s): under torchrun each rank is one client on its
           own GPU (collective FedAvg over RCCL); alone with ``--transport tcp
           --client-index k`` it is the reference's ``python clientK.py``
  server   the reference's ``python server.py``: TCP gather -> FedAvg -> broadcast
  launch   spawn N local ranks (torch.distributed.run, 127.0.0.1) running ``client``
  virtual  N federated clients x R FedAvg rounds in ONE process on one device, trained in turn
           (BASELINE.json config 4's protocol on a single GPU): per-round CSVs + virtual_report.json
  predict  classify every row of a CICIDS2017-format CSV with a trained checkpoint (serving path:
           unpadded HIP forward replayed from HIP graphs); writes probabilities + labels
  bench    the headline benchmark (bench.py)
  scaling  run bench.py at several GPU counts and write the scaling curve
  gen-data write a synthetic CICIDS2017-shaped CSV
  tokenize print WordPiece tokens of a text
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

from .config import FedConfig

PKG = __package__
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _client(argv):
    ap = argparse.ArgumentParser(prog="client")
    FedConfig.add_cli(ap)
    ap.add_argument("--client-index", type=int, default=None, help="0-based client index (tcp mode)")
    ap.add_argument("--layers", type=int, default=None, help="override DistilBERT depth (tests)")
    ns = ap.parse_args(argv)
    cfg = FedConfig.from_args(ns)
    if ns.client_index is not None:
        os.environ["RANK"] = str(ns.client_index)
        os.environ["WORLD_SIZE"] = "1"
        os.environ.setdefault("LOCAL_RANK", "0")
        if cfg.num_clients is None:
            cfg.num_clients = 2
    from .fed.runner import FederatedClient
    from .models import DistilBertConfig
    mc = DistilBertConfig() if ns.layers is None else DistilBertConfig(n_layers=ns.layers)
    client = FederatedClient(cfg, model_config=mc)
    if ns.client_index is not None:  # tcp mode: rank 0 of a 1-process group, identity from the flag
        client.idx, client.client_id = ns.client_index, ns.client_index + 1
        client.log.tag, client.log.name = f"[CLIENT {client.client_id}]", f"Client {client.client_id}"
    rep = client.run()
    print(json.dumps(rep))


def _server(argv):
    ap = argparse.ArgumentParser(prog="server")
    ap.add_argument("--num-clients", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--host", default="localhost")
    ap.add_argument("--port-receive", type=int, default=12345)
    ap.add_argument("--port-send", type=int, default=12346)
    ap.add_argument("--timeout", type=float, default=300.0)
    ap.add_argument("--out-dir", default=".")
    ap.add_argument("--strict-compat", action="store_true",
                    help="drop the GET handshake on downloads (the reference's framing); the payload codec "
                         "stays gzip(torch.save) + weights-only load, so reference pickle clients cannot connect")
    ap.add_argument("--gzip-level", type=int, default=1)
    ns = ap.parse_args(argv)
    from .parallel.transport import FedAvgServer
    from .utils.logging import TagLogger
    log = TagLogger.for_server()
    log.phase("Server starting")
    for r in range(ns.rounds):
        srv = FedAvgServer(ns.num_clients, ns.host, ns.port_receive, ns.port_send, ns.timeout, ns.strict_compat,
                           save_path=os.path.join(ns.out_dir, "ddos_distilbert_model.pth"), log=log,
                           level=ns.gzip_level)
        log.phase(f"Round {r + 1}: waiting for {ns.num_clients} clients")
        if srv.run_round() is None:
            sys.exit(1)
    log.phase("Server shutdown")


def _launch(argv):
    ap = argparse.ArgumentParser(prog="launch")
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--port", type=int, default=29511)
    ap.add_argument("--max-restarts", type=int, default=0,
                    help="elastic recovery: restart the group this many times; clients resume at the "
                         "first unfinished round")
    ns, rest = ap.parse_known_args(argv)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ns.nproc}",
           f"--max-restarts={ns.max_restarts}", "--master-addr", "127.0.0.1", "--master-port", str(ns.port),
           "-m", PKG, "client"] + rest
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.exit(subprocess.call(cmd, env=env))


def _virtual(argv):
    """``--clients N`` virtual clients x ``--rounds R`` (fed/runner.py run_virtual_clients): client k
    samples its own 10 % with seed 42 + k, every round starts from the previous aggregate with a
    fresh Adam, the aggregate is the unweighted mean (server.py:67-79) and every client evaluates it
    on its own test split.  Writes clientK_{local,aggregated}_metrics[_roundR].csv (run_round's
    names), the final aggregate ddos_distilbert_model.pth (+ its round tag) and virtual_report.json."""
    ap = argparse.ArgumentParser(prog="virtual")
    FedConfig.add_cli(ap)
    ap.add_argument("--clients", type=int, default=2)
    ap.add_argument("--layers", type=int, default=None, help="override DistilBERT depth (tests)")
    ap.add_argument("--warm-start-epochs", type=int, default=0,
                    help="train the shared init on a separate public synthetic file first (fed/runner.py "
                         "warm_start: the analog of the reference's pretrained start)")
    ns = ap.parse_args(argv)
    cfg = FedConfig.from_args(ns)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):  # one process, whatever launched it
        os.environ.pop(k, None)
    from .fed.runner import FederatedClient, run_virtual_clients, warm_start
    from .models import DistilBertConfig
    from .utils import checkpoint as ck
    from .utils.metrics import save_metrics
    mc = DistilBertConfig() if ns.layers is None else DistilBertConfig(n_layers=ns.layers)
    cfg.num_clients = ns.clients
    client = FederatedClient(cfg, model_config=mc)
    client.setup()
    log = client.log
    warm = None
    if ns.warm_start_epochs > 0:
        warm = warm_start(client, ns.warm_start_epochs, rows=cfg.synthetic_rows)
        log.info(f"warm start: {ns.warm_start_epochs} epoch(s) on a public synthetic file, public test "
                 f"accuracy {warm['public_test']['accuracy']:.3f} %")
    res = run_virtual_clients(client, ns.clients, rounds=cfg.rounds, progress=log.info)
    os.makedirs(cfg.out_dir, exist_ok=True)

    def tup(m):
        return (m["accuracy"], m["loss"], m["precision"], m["recall"], m["f1"])

    report = {"clients": ns.clients, "rounds": [],
              **({"warm_start": {"epochs": ns.warm_start_epochs, "public_test": warm["public_test"]}} if warm else {})}
    for h in res["rounds"]:
        r = h["round"]
        sfx = "" if r == 1 else f"_round{r}"
        for c in h["clients"]:
            k = c["client"]
            save_metrics(tup(c["local_test"]), os.path.join(cfg.out_dir, f"client{k}_local_metrics{sfx}.csv"))
            save_metrics(tup(c["aggregated_test"]), os.path.join(cfg.out_dir, f"client{k}_aggregated_metrics{sfx}.csv"))
        (tn, fp), (fn, tp) = h["aggregated_confusion"]
        report["rounds"].append({
            "round": r, "fedavg_ms": h["fedavg_ms"], "aggregated_confusion": h["aggregated_confusion"],
            "aggregated_accuracy": 100.0 * (tp + tn) / max(tp + tn + fp + fn, 1),
            "clients": [{"client": c["client"], "local_test": c["local_test"], "aggregated_test": c["aggregated_test"],
                         "epoch_losses": c["train"]["epoch_losses"], "train_steps": c["train"]["steps"],
                         "rel_l2_local_to_aggregate": c["rel_l2_local_to_aggregate"],
                         **({"teacher_test": c["teacher_test"]} if "teacher_test" in c else {})}
                        for c in h["clients"]]})
    if cfg.save_checkpoints:
        ck.save_global(client.model, cfg.out_dir, cfg.rounds)
    path = os.path.join(cfg.out_dir, "virtual_report.json")
    with open(path, "w") as f:
        json.dump(report, f, indent=1)
    log.info(f"virtual federated report written to {path}")
    print(json.dumps({"report": path, "rounds": [
        {"round": r["round"], "aggregated_accuracy": round(r["aggregated_accuracy"], 4)} for r in report["rounds"]]}))


def _predict(argv):
    ap = argparse.ArgumentParser(prog="predict")
    ap.add_argument("--checkpoint", required=True, help="clientN_model.pth / ddos_distilbert_model.pth")
    ap.add_argument("--csv", default=None, help="CICIDS2017-format CSV (default: synthetic rows)")
    ap.add_argument("--rows", type=int, default=20000, help="synthetic rows when --csv is not given")
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--max-len", type=int, default=128)
    ap.add_argument("--out", default="predictions.csv")
    ap.add_argument("--no-graph", action="store_true")
    ns = ap.parse_args(argv)
    import numpy as np
    import pandas as pd
    import torch
    from .data import CICIDS2017Dataset, DeviceLoader, WordPieceTokenizer, generate_cicids2017
    from .data.featurize import clean_frame, render_texts
    from .engine import predict
    from .models import DDoSClassifier
    from .utils.checkpoint import load_model
    from .utils.metrics import binary_prf
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    frame = pd.read_csv(ns.csv) if ns.csv else generate_cicids2017(ns.rows, seed=7)
    frame = clean_frame(frame)
    texts = render_texts(frame)
    has_label = "Label" in frame.columns
    labels = (frame["Label"].to_numpy() == "DDoS").astype(np.int64) if has_label else np.zeros(len(frame), np.int64)
    ds = CICIDS2017Dataset(texts, labels.tolist(), WordPieceTokenizer(), ns.max_len)
    model = DDoSClassifier(device=dev)
    if not load_model(model, ns.checkpoint):
        raise SystemExit(f"cannot load {ns.checkpoint}")
    probs, preds, timing = predict(model, DeviceLoader(ds, ns.batch_size, device=dev), graphed=not ns.no_graph)
    out = pd.DataFrame({"row": np.arange(len(preds)), "prob_ddos": probs, "pred": preds})
    if has_label:
        out["label"] = labels
        tp = int(((preds == 1) & (labels == 1)).sum())
        fp = int(((preds == 1) & (labels == 0)).sum())
        fn = int(((preds == 0) & (labels == 1)).sum())
        p_, r_, f1 = binary_prf(tp, fp, fn)
        timing.update(accuracy=float(100.0 * (preds == labels).mean()), precision=p_, recall=r_, f1=f1)
    out.to_csv(ns.out, index=False)
    print(json.dumps({"out": ns.out, **timing}))


def _bench(argv):
    sys.exit(subprocess.call([sys.executable, os.path.join(ROOT, "bench.py")] + argv))


def _scaling(argv):
    """bench.py at each GPU count, back to back (bench.py starts its own ranks for N > 1, on a
    free rendezvous port); unknown arguments are passed to every bench run."""
    ap = argparse.ArgumentParser(prog="scaling")
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--out", default="scaling.json")
    ns, extra = ap.parse_known_args(argv)
    results = []
    for n in (int(x) for x in ns.gpus.split(",")):
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", str(ns.steps),
               "--warmup", str(ns.warmup)] + extra
        env = dict(os.environ)
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):  # bench.py launches its own ranks
            env.pop(k, None)
        out = subprocess.run(cmd, capture_output=True, text=True, env=env)
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        if not line:
            print(out.stdout[-2000:], out.stderr[-2000:], file=sys.stderr)
            continue
        results.append(json.loads(line[-1]))
        print(line[-1], flush=True)
    if results:
        base = results[0]["per_client_batches_per_sec"]
        for r in results:
            r["per_client_efficiency_vs_1gpu"] = round(r["per_client_batches_per_sec"] / base, 4)
        # per-step time and FedAvg round time side by side (bench.py times them apart: the step
        # window holds local steps only, the round -- one per 2,541 reference steps -- its own)
        print(f"{'gpus':>4} {'ms/step':>9} {'batches/s/client':>17} {'eff':>6} {'fedavg round ms':>16} "
              f"{'all-reduce GB/s':>16} {'ms/step incl. round':>20}")
        for r in results:
            fr, bw, inc = r.get("fedavg_round_ms"), r.get("allreduce_busbw_GBps"), r.get("ms_per_step_incl_round")
            print(f"{r['n_gpus']:>4} {r['ms_per_step']:>9.4f} {r['per_client_batches_per_sec']:>17.2f} "
                  f"{r['per_client_efficiency_vs_1gpu']:>6.3f} {'-' if fr is None else f'{fr:.3f}':>16} "
                  f"{'-' if bw is None else f'{bw:.1f}':>16} {'-' if inc is None else f'{inc:.4f}':>20}")
        with open(ns.out, "w") as f:
            json.dump(results, f, indent=1)
        from .utils.plots import plot_scaling
        plot_scaling(results, os.path.splitext(ns.out)[0] + ".png")


def _gen_data(argv):
    ap = argparse.ArgumentParser(prog="gen-data")
    ap.add_argument("--rows", type=int, default=225_745)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="CICIDS2017.csv")
    ns = ap.parse_args(argv)
    from .data.synthetic import generate_cicids2017, write_csv
    write_csv(generate_cicids2017(ns.rows, ns.seed), ns.out)
    print(ns.out)


def _tokenize(argv):
    from .data.tokenizer import WordPieceTokenizer
    tok = WordPieceTokenizer()
    text = " ".join(argv)
    print(tok.tokenize(text))
    print(tok(text, max_length=128)["input_ids"])


COMMANDS = {"client": _client, "server": _server, "launch": _launch, "virtual": _virtual, "predict": _predict,
            "bench": _bench,
            "scaling": _scaling,
            "gen-data": _gen_data, "tokenize": _tokenize}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in COMMANDS:
        print(__doc__)
        sys.exit(0 if not argv else 2)
    COMMANDS[argv[0]](argv[1:])


if __name__ == "__main__":
    main()

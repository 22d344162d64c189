"""Command line (the reference's process entrypoint, index.js:1-40, plus operational tools).

  python -m downloader_amd worker      [--config F]   consume v1.download (index.js init())
  python -m downloader_amd supervisor  -n 8           N workers on one host, auto-restart
  python -m downloader_amd broker      [--port 5672]  bundled AMQP 0-9-1 broker
  python -m downloader_amd submit      ID SOURCE URI [--type TV]   publish an api.Download
  python -m downloader_amd make-torrent PATH -o F [--webseed URL] [--tracker URL]
  python -m downloader_amd verify      TORRENT DIR [--backend gpu|cpu|auto]
  python -m downloader_amd config                     print the effective config
  python -m downloader_amd doctor      [--sharers N]  host readiness report (JSON + warnings)

Worker lifecycle mirrors index.js: logger + tracer, load config (named ``downloader``; the
reference's ``'converter'`` is accepted as an alias), start the service, and on SIGINT/SIGTERM
or an unhandled error run the termination handler and exit 0 when idle / 1 when jobs were in
flight (lib/main.js:197-204; App. A #2 fixed so that "idle" is real).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import signal
import sys
import time

from .utils.cpus import effective_cpus


def _worker(args) -> int:
    from .service.worker import Worker
    from .utils.config import load_config
    from .utils.log import get_logger
    log = get_logger("index.py")
    from .utils.limits import raise_nofile
    cfg = load_config(path=args.config or None)
    if args.mode:
        cfg.mode = args.mode
        cfg.apply_mode()
    raise_nofile()   # one descriptor per torrent file for a session: EMFILE at 1,024 otherwise

    async def main() -> int:
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for sig in (signal.SIGINT, signal.SIGTERM):   # before start(): no startup window
            loop.add_signal_handler(sig, stop.set)
        w = Worker(cfg, logger=get_logger("main"))
        await w.start()
        log.info("initialized")

        def on_error(loop, ctx):
            log.error("Unhandled exception", str(ctx.get("exception") or ctx.get("message")))
            stop.set()
        loop.set_exception_handler(on_error)
        await stop.wait()
        code = await w.stop(drain_timeout=args.drain_timeout)
        log.info("exiting", code=code)
        return code
    return asyncio.run(main())


def _supervisor(args) -> int:
    from .parallel.supervisor import Supervisor, worker_argv
    extra = ["--mode", args.mode] if args.mode else []
    sup = Supervisor(args.n, worker_argv(args.config, extra), cpus_per_worker=args.cpus_per_worker,
                     base_port=args.base_port)
    return sup.run_forever()


def _broker(args) -> int:
    from .broker.server import run_broker
    try:
        asyncio.run(run_broker(args.host, args.port, args.consumer_timeout, args.certfile,
                               args.keyfile, args.client_ca))
    except KeyboardInterrupt:
        pass
    return 0


def _submit(args) -> int:
    from .broker.amqp import AmqpBroker
    from .models import api
    from .utils.config import load_config
    from .utils.dynamics import dyn
    cfg = load_config(path=args.config or None)

    async def main() -> None:
        b = AmqpBroker(cfg.broker.url or dyn("rabbitmq"))
        await b.connect()
        msg = api.make_download(args.id, args.source, args.uri, args.type, args.creator)
        await b.publish(cfg.broker.download_queue, api.encode(msg))
        await b.close()
    asyncio.run(main())
    return 0


def _make_torrent(args) -> int:
    from .torrent.metainfo import make_torrent, parse_torrent
    raw = make_torrent(args.path, args.piece_length, args.tracker or [], args.webseed or [])
    with open(args.output, "wb") as f:
        f.write(raw)
    m = parse_torrent(raw)
    print(json.dumps({"info_hash": m.info_hash.hex(), "pieces": m.num_pieces,
                      "piece_length": m.piece_length, "bytes": m.total_length}))
    return 0


def _verify(args) -> int:
    from .ops import hashing
    from .torrent.metainfo import parse_torrent
    with open(args.torrent, "rb") as f:
        m = parse_torrent(f.read())
    files = m.local_files(args.dir)
    t0 = time.perf_counter()
    ok = hashing.verify_pieces(files, m.piece_length, m.pieces, backend=args.backend)
    dt = time.perf_counter() - t0
    good = sum(ok)
    print(json.dumps({"pieces": len(ok), "good": good, "seconds": round(dt, 4),
                      "GBps": round(m.total_length / dt / 1e9, 3) if dt else None,
                      "backend": hashing.choose_backend(args.backend, m.total_length, len(ok))}))
    return 0 if good == len(ok) else 1


def _config(args) -> int:
    """Print the effective config. Secrets (S3 secret key, broker URL password) are masked
    unless ``--show-secrets`` (App. A #19: the reference logged bucket:// credentials)."""
    from urllib.parse import urlsplit, urlunsplit

    from .utils.config import load_config
    if args.reference:
        from .utils.config_doc import reference_markdown
        print(reference_markdown())
        return 0
    d = load_config(path=args.config or None).model_dump(mode="json")
    if not args.show_secrets:
        for k in ("secret_key", "session_token"):
            if d.get("s3", {}).get(k):
                d["s3"][k] = "***"
        url = d.get("broker", {}).get("url") or ""
        u = urlsplit(url)
        if u.password:
            netloc = f"{u.username}:***@{u.hostname}" + (f":{u.port}" if u.port else "")
            d["broker"]["url"] = urlunsplit(u._replace(netloc=netloc))
    print(json.dumps(d, indent=2))
    return 0


def _doctor(args) -> int:
    from .utils.doctor import report
    print(json.dumps(report(args.sharers), indent=2))
    return 0


def main(argv=None) -> int:
    p = argparse.ArgumentParser(prog="downloader_amd")
    sub = p.add_subparsers(dest="cmd", required=True)
    w = sub.add_parser("worker")
    w.add_argument("--config", default="")
    w.add_argument("--mode", choices=["tuned", "reference"], default="")
    w.add_argument("--drain-timeout", type=float, default=30.0)
    s = sub.add_parser("supervisor")
    # one worker (4 jobs in flight, native threads for hashing/relay) per 4 usable CPUs
    s.add_argument("-n", type=int, default=max(1, effective_cpus() // 4))
    s.add_argument("--config", default="")
    s.add_argument("--mode", choices=["tuned", "reference"], default="")
    s.add_argument("--cpus-per-worker", type=int, default=0,
                   help="K: pin each worker to K CPUs; 0: share of the cgroup quota; -1: off")
    s.add_argument("--base-port", type=int, default=0)
    b = sub.add_parser("broker")
    b.add_argument("--host", default="0.0.0.0")
    b.add_argument("--port", type=int, default=5672)
    b.add_argument("--consumer-timeout", type=float, default=0.0,
                   help="close a channel whose delivery stays unacked this long (s, 0: never)")
    b.add_argument("--certfile", default="", help="PEM certificate: serve amqps://")
    b.add_argument("--keyfile", default="")
    b.add_argument("--client-ca", default="",
                   help="PEM CA: require client certificates from it (mutual TLS)")
    su = sub.add_parser("submit")
    su.add_argument("id")
    su.add_argument("source", choices=["http", "torrent", "file", "bucket"])
    su.add_argument("uri")
    su.add_argument("--type", default="MOVIE", choices=["MOVIE", "TV"])
    su.add_argument("--creator", default="")
    su.add_argument("--config", default="")
    mt = sub.add_parser("make-torrent")
    mt.add_argument("path")
    mt.add_argument("-o", "--output", required=True)
    mt.add_argument("--piece-length", type=int, default=0)
    mt.add_argument("--tracker", action="append")
    mt.add_argument("--webseed", action="append")
    v = sub.add_parser("verify")
    v.add_argument("torrent")
    v.add_argument("dir")
    v.add_argument("--backend", default="auto", choices=["auto", "cpu", "gpu"])
    c = sub.add_parser("config")
    c.add_argument("--config", default="")
    c.add_argument("--show-secrets", action="store_true", help="do not mask credentials")
    c.add_argument("--reference", action="store_true",
                   help="print the markdown reference of every key (docs/CONFIG.md)")
    d = sub.add_parser("doctor")
    d.add_argument("--sharers", type=int, default=4,
                   help="worker processes of this uid per host (they share the pipe budget)")
    args = p.parse_args(argv)
    return {"worker": _worker, "supervisor": _supervisor, "broker": _broker, "submit": _submit,
            "make-torrent": _make_torrent, "verify": _verify, "config": _config,
            "doctor": _doctor}[args.cmd](args)


if __name__ == "__main__":
    sys.exit(main())

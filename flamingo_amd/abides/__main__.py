"""Entry point with the reference's two-stage flag parsing (abides.py:17-29):
``python -m flamingo_amd.abides -c flamingo [config flags]``."""
import argparse
import sys

BANNER = "ABIDES: Agent-Based Interactive Discrete Event Simulation"


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    print("=" * (len(BANNER) + 2))
    print(" " + BANNER)
    print("=" * (len(BANNER) + 2))
    print()
    ap = argparse.ArgumentParser(description="Simulation configuration.")
    ap.add_argument("-c", "--config", required=True)
    ap.add_argument("--config-help", action="store_true")
    args, _ = ap.parse_known_args(argv)
    if args.config != "flamingo":
        raise SystemExit(f"config {args.config!r} is not part of this repository (only 'flamingo')")
    from .config_flamingo import run
    from .flamingo import protocol
    res = run(argv)
    # explicit teardown (the server's store, its device group and RCCL clique, the engine) instead of
    # leaving them to finalizers at interpreter exit
    if res is not None:
        srv = res.get("server")
        if srv is not None and srv._store is not None:
            srv._store.close()
    protocol.shutdown()


if __name__ == "__main__":
    main()

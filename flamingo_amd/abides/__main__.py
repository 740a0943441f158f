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
    run(argv)


if __name__ == "__main__":
    main()

"""Verbosity switch shared by the simulation (util/util.py:14-23 surface)."""
silent_mode = False


def log_print(fmt, *args):
    if not silent_mode:
        print(fmt.format(*args))


def be_silent():
    return silent_mode

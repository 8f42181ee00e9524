"""gflags-style command-line flags (replacement for ``tf.app.flags``).

The reference defines its CLI with ``tf.app.flags.DEFINE_*`` at module import
time and parses ``sys.argv`` inside ``tf.app.run()`` (``main.py:10-32,161-162``,
``inference.py:14-30,115-116``).  Flags are process-global and shared between
modules (``mnist_input.py:9`` reaches the same ``FLAGS`` object).

This module reproduces that surface so existing launch lines keep working:

* ``--name=value`` and ``--name value`` forms;
* booleans accept ``--name``, ``--noname``, ``--name=true|false|1|0``;
* unknown flags raise (gflags behaviour) unless ``allow_unknown=True``;
* ``FLAGS.name`` attribute access, assignable (``main.py:66`` assigns
  ``FLAGS.task_id = 0``).
"""
from __future__ import annotations

import sys
from typing import Any, Callable, Dict, List, Optional


class FlagError(ValueError):
    pass


def _parse_bool(v: str) -> bool:
    s = str(v).strip().lower()
    if s in ("1", "true", "t", "yes", "y", "on"):
        return True
    if s in ("0", "false", "f", "no", "n", "off"):
        return False
    raise FlagError(f"invalid boolean value {v!r}")


class _Flag:
    __slots__ = ("name", "default", "help", "parser", "kind", "value", "present")

    def __init__(self, name: str, default: Any, help: str, parser: Callable[[str], Any], kind: str):
        self.name = name
        self.default = default
        self.help = help
        self.parser = parser
        self.kind = kind
        self.value = default
        self.present = False


class FlagValues:
    """Registry + parsed values.  One global instance: ``FLAGS``."""

    def __init__(self) -> None:
        object.__setattr__(self, "_flags", {})
        object.__setattr__(self, "_parsed", False)

    # -- definition -----------------------------------------------------
    def _define(self, name: str, default: Any, help: str, parser: Callable[[str], Any], kind: str) -> None:
        flags: Dict[str, _Flag] = self._flags
        if name in flags:
            # Re-definition with the same kind is tolerated (module reloads in tests).
            if flags[name].kind != kind:
                raise FlagError(f"flag {name!r} redefined with a different type")
            return
        flags[name] = _Flag(name, default, help, parser, kind)

    # -- access ----------------------------------------------------------
    def __getattr__(self, name: str) -> Any:
        flags = object.__getattribute__(self, "_flags")
        if name in flags:
            return flags[name].value
        raise AttributeError(name)

    def __setattr__(self, name: str, value: Any) -> None:
        flags = self._flags
        if name not in flags:
            raise AttributeError(f"unknown flag {name!r}")
        flags[name].value = value

    def __contains__(self, name: str) -> bool:
        return name in self._flags

    def is_present(self, name: str) -> bool:
        return self._flags[name].present

    def flag_dict(self) -> Dict[str, Any]:
        return {k: f.value for k, f in self._flags.items()}

    def reset(self) -> None:
        for f in self._flags.values():
            f.value = f.default
            f.present = False
        object.__setattr__(self, "_parsed", False)

    # -- parsing ---------------------------------------------------------
    def parse(self, argv: List[str], allow_unknown: bool = False) -> List[str]:
        """Parse ``argv`` (without the program name).  Returns leftover args."""
        flags: Dict[str, _Flag] = self._flags
        rest: List[str] = []
        i = 0
        while i < len(argv):
            a = argv[i]
            if a == "--":
                rest.extend(argv[i + 1:])
                break
            if not a.startswith("-") or a == "-":
                rest.append(a)
                i += 1
                continue
            body = a.lstrip("-")
            if "=" in body:
                name, val = body.split("=", 1)
                has_val = True
            else:
                name, val, has_val = body, None, False
            name = name.replace("-", "_")
            f = flags.get(name)
            if f is None and name.startswith("no") and name[2:] in flags and flags[name[2:]].kind == "bool" and not has_val:
                f = flags[name[2:]]
                f.value = False
                f.present = True
                i += 1
                continue
            if f is None:
                if name in ("help", "h", "helpfull"):
                    print(self.usage())
                    raise SystemExit(0)
                if allow_unknown:
                    rest.append(a)
                    i += 1
                    continue
                raise FlagError(f"unknown command line flag {name!r}")
            if f.kind == "bool":
                f.value = True if not has_val else _parse_bool(val)
            else:
                if not has_val:
                    if i + 1 >= len(argv):
                        raise FlagError(f"flag --{name} needs a value")
                    val = argv[i + 1]
                    i += 1
                try:
                    f.value = f.parser(val)
                except (TypeError, ValueError) as e:
                    raise FlagError(f"bad value for --{name}: {val!r} ({e})") from e
            f.present = True
            i += 1
        object.__setattr__(self, "_parsed", True)
        return rest

    def usage(self) -> str:
        lines = ["flags:"]
        for f in sorted(self._flags.values(), key=lambda x: x.name):
            lines.append(f"  --{f.name} ({f.kind}, default {f.default!r}): {f.help}")
        return "\n".join(lines)


FLAGS = FlagValues()


def DEFINE_string(name: str, default: Optional[str], help: str = "") -> None:
    FLAGS._define(name, default, help, str, "string")


def DEFINE_integer(name: str, default: Optional[int], help: str = "") -> None:
    FLAGS._define(name, default, help, lambda v: int(v, 0) if isinstance(v, str) else int(v), "int")


def DEFINE_float(name: str, default: Optional[float], help: str = "") -> None:
    FLAGS._define(name, default, help, float, "float")


def DEFINE_boolean(name: str, default: bool, help: str = "") -> None:
    FLAGS._define(name, default, help, _parse_bool, "bool")


DEFINE_bool = DEFINE_boolean


def run(main: Callable[[List[str]], Any], argv: Optional[List[str]] = None) -> None:
    """``tf.app.run`` equivalent: parse flags, call ``main(argv)``, exit with its code."""
    argv = list(sys.argv if argv is None else argv)
    rest = FLAGS.parse(argv[1:])
    rc = main([argv[0]] + rest)
    sys.exit(rc if isinstance(rc, int) else 0)

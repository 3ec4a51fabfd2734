"""Go ``flag`` package semantics, re-implemented for the autoscaler CLI.

The reference's whole configuration surface is Go's ``flag`` package (/root/reference/main.go:83-99):
``-name=value``, ``--name=value`` and ``-name value``; parsing stops at the first non-flag
argument or after ``--``; ints parse with ``strconv.ParseInt(s, 0, 64)`` (so ``0x10``, ``010``,
``0b1``, ``1_000`` work); durations parse with ``time.ParseDuration``; a bad value prints
``invalid value "x" for flag -name: parse error`` plus the usage text and exits 2; ``-h`` /
``-help`` print usage and exit 0 (Go >= 1.15, the reference's toolchain, .travis.yml:4).
Usage text follows ``flag.PrintDefaults`` byte for byte so operators see the same help.
"""
from __future__ import annotations

import sys
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, TextIO

INT64_MIN = -(1 << 63)
INT64_MAX = (1 << 63) - 1

NANOSECOND = 1
MICROSECOND = 1000
MILLISECOND = 1000 * MICROSECOND
SECOND = 1000 * MILLISECOND
MINUTE = 60 * SECOND
HOUR = 60 * MINUTE


class GoSyntaxError(ValueError):
    """strconv.ErrSyntax / time.ParseDuration failure."""


class GoRangeError(ValueError):
    """strconv.ErrRange."""


# ---------------------------------------------------------------------------------------------
# strconv.ParseInt(s, 0, 64)


def _underscore_ok(s: str) -> bool:
    """strconv.underscoreOK: '_' only between digits or between a base prefix and a digit."""
    saw = "^"
    i = 0
    if len(s) >= 1 and s[0] in "+-":
        s = s[1:]
    hexa = False
    if len(s) >= 2 and s[0] == "0" and s[1].lower() in "box":
        i = 2
        saw = "0"
        hexa = s[1].lower() == "x"
    while i < len(s):
        c = s[i]
        i += 1
        if "0" <= c <= "9" or (hexa and "a" <= c.lower() <= "f"):
            saw = "0"
            continue
        if c == "_":
            if saw != "0":
                return False
            saw = "_"
            continue
        if saw == "_":
            return False
        saw = "!"
    return saw != "_"


def parse_int(s: str, bit_size: int = 64) -> int:
    """strconv.ParseInt(s, 0, bit_size): sign, base prefixes 0b/0o/0x/0, '_' separators."""
    s0 = s

    def syntax() -> GoSyntaxError:
        return GoSyntaxError(f'strconv.ParseInt: parsing "{s0}": invalid syntax')

    def rng() -> GoRangeError:
        return GoRangeError(f'strconv.ParseInt: parsing "{s0}": value out of range')

    if s == "":
        raise syntax()
    neg = False
    if s[0] in "+-":
        neg = s[0] == "-"
        s = s[1:]
    # strconv.ParseUint(s, 0, bit_size)
    if s == "":
        raise syntax()
    base = 10
    if s[0] == "0":
        if len(s) >= 3 and s[1].lower() == "b":
            base, s = 2, s[2:]
        elif len(s) >= 3 and s[1].lower() == "o":
            base, s = 8, s[2:]
        elif len(s) >= 3 and s[1].lower() == "x":
            base, s = 16, s[2:]
        else:
            base, s = 8, s[1:]
    max_val = (1 << 64) - 1
    n = 0
    underscores = False
    for c in s:
        if c == "_":
            underscores = True
            continue
        if "0" <= c <= "9":
            d = ord(c) - 48
        elif "a" <= c.lower() <= "z":
            d = ord(c.lower()) - ord("a") + 10
        else:
            raise syntax()
        if d >= base:
            raise syntax()
        n = n * base + d
        if n > max_val:
            raise rng()
    if underscores and not _underscore_ok(s0):
        raise syntax()
    cutoff = 1 << (bit_size - 1)
    if not neg and n >= cutoff:
        raise rng()
    if neg and n > cutoff:
        raise rng()
    return -n if neg else n


# ---------------------------------------------------------------------------------------------
# time.ParseDuration / Duration.String

_UNITS = {
    "ns": NANOSECOND,
    "us": MICROSECOND,
    "µs": MICROSECOND,  # U+00B5 micro sign
    "μs": MICROSECOND,  # U+03BC greek mu
    "ms": MILLISECOND,
    "s": SECOND,
    "m": MINUTE,
    "h": HOUR,
}


def parse_duration(s: str) -> int:
    """time.ParseDuration -> nanoseconds (int64). Raises GoSyntaxError with Go's messages."""
    orig = s
    quoted = '"' + orig + '"'
    d = 0
    neg = False
    if s and s[0] in "-+":
        neg = s[0] == "-"
        s = s[1:]
    if s == "0":
        return 0
    if s == "":
        raise GoSyntaxError("time: invalid duration " + quoted)
    while s:
        # integer part
        i = 0
        while i < len(s) and "0" <= s[i] <= "9":
            i += 1
        int_part = s[:i]
        pre = i > 0
        s = s[i:]
        frac_part = ""
        post = False
        if s and s[0] == ".":
            s = s[1:]
            j = 0
            while j < len(s) and "0" <= s[j] <= "9":
                j += 1
            frac_part = s[:j]
            post = j > 0
            s = s[j:]
        if not pre and not post:
            raise GoSyntaxError("time: invalid duration " + quoted)
        k = 0
        while k < len(s) and s[k] != "." and not ("0" <= s[k] <= "9"):
            k += 1
        if k == 0:
            raise GoSyntaxError("time: missing unit in duration " + quoted)
        u = s[:k]
        s = s[k:]
        if u not in _UNITS:
            raise GoSyntaxError('time: unknown unit "' + u + '" in duration ' + quoted)
        unit = _UNITS[u]
        v = int(int_part) if int_part else 0
        if v > (1 << 63) // unit:
            raise GoSyntaxError("time: invalid duration " + quoted)
        v *= unit
        if frac_part:
            # Go accumulates the fraction with float64 scaling, truncated toward zero.
            f = 0
            scale = 1
            for c in frac_part:
                if f > (1 << 63) // 10:  # overflow: ignore further digits like Go
                    break
                f = f * 10 + ord(c) - 48
                scale *= 10
            v += int(float(f) * (float(unit) / float(scale)))
            if v > (1 << 63):
                raise GoSyntaxError("time: invalid duration " + quoted)
        d += v
        if d > (1 << 63):
            raise GoSyntaxError("time: invalid duration " + quoted)
    if neg:
        return -d
    if d > INT64_MAX:
        raise GoSyntaxError("time: invalid duration " + quoted)
    return d


def parse_float(s: str) -> float:
    """strconv.ParseFloat(s, 64): decimal or hex (``0x1p-2``) literals, ``_`` between digits,
    ``inf``/``infinity``/``nan`` in any case; no surrounding space. Overflow is ErrRange."""
    s0 = s

    def syntax() -> GoSyntaxError:
        return GoSyntaxError(f'strconv.ParseFloat: parsing "{s0}": invalid syntax')

    if not s or not s.isascii() or s != s.strip():
        raise syntax()
    neg = s[0] == "-"
    body = s[1:] if s[0] in "+-" else s
    special = body.lower()
    if special in ("inf", "infinity"):
        return float("-inf") if neg else float("inf")
    if special == "nan":
        if body != s:  # Go accepts no sign on NaN
            raise syntax()
        return float("nan")
    if "_" in s:
        if not _underscore_ok(s):
            raise syntax()
        s = s.replace("_", "")
        body = s[1:] if s[0] in "+-" else s
    hexa = body[:2].lower() == "0x"
    if hexa:
        if "p" not in body.lower():  # Go requires the binary exponent on hex floats
            raise syntax()
        try:
            v = float.fromhex(s)
        except OverflowError:
            raise GoRangeError(f'strconv.ParseFloat: parsing "{s0}": value out of range')
        except ValueError:
            raise syntax()
    else:
        if any(c not in "0123456789.eE+-" for c in body) or not any(c.isdigit() for c in body):
            raise syntax()
        try:
            v = float(s)
        except ValueError:
            raise syntax()
    if v in (float("inf"), float("-inf")):
        raise GoRangeError(f'strconv.ParseFloat: parsing "{s0}": value out of range')
    return v


def format_float(v: float) -> str:
    """strconv.FormatFloat(v, 'g', -1, 64) -- flag.Float64's String(): shortest round-trip
    digits, %e form when the decimal exponent is < -4 or >= 6 (eprec is 6 for shortest)."""
    import math
    from decimal import Decimal

    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    if v == 0:
        return "-0" if math.copysign(1.0, v) < 0 else "0"
    sign, digits, exp10 = Decimal(repr(v)).normalize().as_tuple()
    ds = "".join(map(str, digits))
    dp = len(ds) + exp10  # position of the decimal point within ds
    exp = dp - 1
    neg = "-" if sign else ""
    if exp < -4 or exp >= 6:
        mant = ds[0] + ("." + ds[1:] if len(ds) > 1 else "")
        return f"{neg}{mant}e{'-' if exp < 0 else '+'}{abs(exp):02d}"
    if dp <= 0:
        return f"{neg}0.{'0' * -dp}{ds}"
    if dp >= len(ds):
        return f"{neg}{ds}{'0' * (dp - len(ds))}"
    return f"{neg}{ds[:dp]}.{ds[dp:]}"


def _fmt_frac(v: int, prec: int) -> tuple[str, int]:
    out = ""
    printed = False
    for _ in range(prec):
        digit = v % 10
        printed = printed or digit != 0
        if printed:
            out = chr(48 + digit) + out
        v //= 10
    if printed:
        out = "." + out
    return out, v


def format_duration(d: int) -> str:
    """time.Duration.String()."""
    if d == 0:
        return "0s"
    neg = d < 0
    u = -d if neg else d
    if u < SECOND:
        if u < MICROSECOND:
            s = f"{u}ns"
        elif u < MILLISECOND:
            frac, whole = _fmt_frac(u, 3)
            s = f"{whole}{frac}µs"
        else:
            frac, whole = _fmt_frac(u, 6)
            s = f"{whole}{frac}ms"
    else:
        frac, whole = _fmt_frac(u, 9)
        secs = whole % 60
        mins_total = whole // 60
        s = f"{secs}{frac}s"
        if mins_total > 0:
            s = f"{mins_total % 60}m" + s
            hours = mins_total // 60
            if hours > 0:
                s = f"{hours}h" + s
    return "-" + s if neg else s


# ---------------------------------------------------------------------------------------------
# FlagSet


class FlagError(Exception):
    """A parse failure; ``str(e)`` is Go's message. ``help`` is set for -h/-help."""

    def __init__(self, msg: str, help: bool = False):
        super().__init__(msg)
        self.help = help


@dataclass
class Flag:
    name: str
    kind: str  # "duration" | "int" | "string" | "bool" | "value"
    default: Any
    usage: str
    setter: Callable[[str], Any]
    formatter: Callable[[Any], str]
    value: Any = None
    repeated: bool = False
    set_count: int = 0

    @property
    def default_text(self) -> str:
        return self.formatter(self.default)

    def is_zero_default(self) -> bool:
        zero = {"duration": "0s", "int": "0", "float": "0", "string": "", "bool": "false", "value": ""}.get(self.kind, "")
        return self.default_text == zero


@dataclass
class FlagSet:
    """flag.FlagSet with ContinueOnError semantics (the CLI maps errors to exit codes)."""

    program: str = "kube-sqs-autoscaler"
    flags: Dict[str, Flag] = field(default_factory=dict)
    args: List[str] = field(default_factory=list)
    order: List[str] = field(default_factory=list)  # names in the order they were set

    # -- definitions ---------------------------------------------------------------------
    def _add(self, f: Flag) -> Flag:
        if f.name in self.flags:
            raise ValueError(f"flag redefined: {f.name}")
        f.value = list(f.default) if f.repeated else f.default
        self.flags[f.name] = f
        return f

    def duration(self, name: str, default_ns: int, usage: str) -> Flag:
        return self._add(Flag(name, "duration", default_ns, usage, parse_duration, format_duration))

    def int(self, name: str, default: int, usage: str) -> Flag:
        return self._add(Flag(name, "int", default, usage, parse_int, str))

    def float64(self, name: str, default: float, usage: str) -> Flag:
        return self._add(Flag(name, "float", default, usage, parse_float, format_float))

    def string(self, name: str, default: str, usage: str) -> Flag:
        return self._add(Flag(name, "string", default, usage, lambda s: s, lambda v: v))

    def bool(self, name: str, default: bool, usage: str) -> Flag:
        def setb(s: str) -> bool:
            # strconv.ParseBool
            if s in ("1", "t", "T", "TRUE", "true", "True"):
                return True
            if s in ("0", "f", "F", "FALSE", "false", "False"):
                return False
            raise GoSyntaxError(f'strconv.ParseBool: parsing "{s}": invalid syntax')

        return self._add(Flag(name, "bool", default, usage, setb, lambda v: "true" if v else "false"))

    def strings(self, name: str, usage: str) -> Flag:
        """Repeatable string flag (a flag.Value that appends); extension-only."""
        return self._add(
            Flag(name, "value", [], usage, lambda s: s, lambda v: ",".join(v) if v else "", repeated=True)
        )

    # -- access ---------------------------------------------------------------------------
    def __getitem__(self, name: str) -> Any:
        return self.flags[name].value

    def was_set(self, name: str) -> bool:
        return self.flags[name].set_count > 0

    # -- parsing (flag.FlagSet.parseOne) --------------------------------------------------
    def parse(self, argv: List[str]) -> None:
        args = list(argv)
        while args:
            s = args[0]
            if len(s) < 2 or s[0] != "-":
                break
            num_minuses = 1
            if s[1] == "-":
                num_minuses = 2
                if len(s) == 2:  # "--" terminates the flags
                    args.pop(0)
                    break
            name = s[num_minuses:]
            if len(name) == 0 or name[0] == "-" or name[0] == "=":
                raise FlagError(f"bad flag syntax: {s}")
            args.pop(0)
            has_value = False
            value = ""
            if "=" in name[1:]:
                i = name.index("=", 1)
                value = name[i + 1 :]
                has_value = True
                name = name[:i]
            f = self.flags.get(name)
            if f is None:
                if name in ("help", "h"):
                    raise FlagError("flag: help requested", help=True)
                raise FlagError(f"flag provided but not defined: -{name}")
            if f.kind == "bool":
                if has_value:
                    try:
                        self._set(f, value)
                    except ValueError:
                        raise FlagError(f'invalid boolean value "{value}" for -{name}: parse error')
                else:
                    self._set(f, "true")
            else:
                if not has_value and args:
                    has_value = True
                    value = args.pop(0)
                if not has_value:
                    raise FlagError(f"flag needs an argument: -{name}")
                try:
                    self._set(f, value)
                except GoRangeError:
                    raise FlagError(f'invalid value "{value}" for flag -{name}: value out of range')
                except ValueError:
                    raise FlagError(f'invalid value "{value}" for flag -{name}: parse error')
        self.args = args

    def _set(self, f: Flag, value: str) -> None:
        v = f.setter(value)
        if f.repeated:
            if f.set_count == 0:
                f.value = []
            f.value.append(v)
        else:
            f.value = v
        f.set_count += 1
        self.order.append(f.name)

    # -- usage (flag.PrintDefaults) -------------------------------------------------------
    def usage(self) -> str:
        out = [f"Usage of {self.program}:\n"]
        for name in sorted(self.flags):
            f = self.flags[name]
            line = "  -" + name
            tname, usage = _unquote_usage(f)
            if tname:
                line += " " + tname
            if len(line) <= 4:
                line += "\t"
            else:
                line += "\n    \t"
            line += usage.replace("\n", "\n    \t")
            if not f.is_zero_default():
                if f.kind == "string":
                    line += f" (default {_go_quote(f.default_text)})"
                else:
                    line += f" (default {f.default_text})"
            out.append(line + "\n")
        return "".join(out)

    def print_usage(self, stream: Optional[TextIO] = None) -> None:
        (stream or sys.stderr).write(self.usage())


def _unquote_usage(f: Flag) -> tuple[str, str]:
    usage = f.usage
    i = usage.find("`")
    if i >= 0:
        j = usage.find("`", i + 1)
        if j >= 0:
            name = usage[i + 1 : j]
            return name, usage[:i] + name + usage[j + 1 :]
    return {"bool": "", "duration": "duration", "int": "int", "float": "float", "string": "string"}.get(f.kind, "value"), usage


def _go_quote(s: str) -> str:
    """strconv.Quote for the printable-ASCII/UTF-8 strings flag defaults contain."""
    out = ['"']
    for ch in s:
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\t":
            out.append("\\t")
        elif ch == "\r":
            out.append("\\r")
        elif ord(ch) < 0x20 or ord(ch) == 0x7F:
            out.append(f"\\x{ord(ch):02x}")
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)

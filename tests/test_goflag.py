"""Go flag / strconv / time.ParseDuration fidelity (reference CLI surface, main.go:83-99)."""
import pytest

from kube_sqs_autoscaler_amd.utils.goflag import (
    HOUR, MILLISECOND, MINUTE, SECOND, FlagError, FlagSet, GoRangeError, GoSyntaxError,
    format_duration, parse_duration, parse_int)


@pytest.mark.parametrize("s,v", [
    ("0", 0), ("7", 7), ("-7", -7), ("+7", 7), ("010", 8), ("0x10", 16), ("0X1f", 31), ("0b101", 5),
    ("0o17", 15), ("0O17", 15), ("1_000", 1000), ("0x_ff", 255), ("0_7", 7), ("00", 0),
    ("9223372036854775807", 2**63 - 1), ("-9223372036854775808", -2**63),
])
def test_parse_int_base0(s, v):
    assert parse_int(s) == v


@pytest.mark.parametrize("s", ["", "-", "+", "0x", "0b", "08", "0b2", "1__0", "_1", "1_", "abc", " 1", "1.0", "0x_", "1e3"])
def test_parse_int_syntax_errors(s):
    with pytest.raises(GoSyntaxError):
        parse_int(s)


@pytest.mark.parametrize("s", ["9223372036854775808", "-9223372036854775809", "0x8000000000000000", "99999999999999999999999"])
def test_parse_int_range_errors(s):
    with pytest.raises(GoRangeError):
        parse_int(s)


@pytest.mark.parametrize("s,ns", [
    ("5s", 5 * SECOND), ("30s", 30 * SECOND), ("5m", 5 * MINUTE), ("1h30m", 90 * MINUTE), ("500ms", 500 * MILLISECOND),
    ("1.5s", 1500 * MILLISECOND), (".5s", 500 * MILLISECOND), ("1.s", SECOND), ("0", 0), ("-0", 0), ("+5s", 5 * SECOND),
    ("-1m", -MINUTE), ("1ns", 1), ("1us", 1000), ("1µs", 1000), ("1μs", 1000), ("2h45m0.5s", 2 * HOUR + 45 * MINUTE + 500 * MILLISECOND),
    ("1h1h", 2 * HOUR), ("0.000000001s", 1), ("2562047h", 2562047 * HOUR),
])
def test_parse_duration(s, ns):
    assert parse_duration(s) == ns


@pytest.mark.parametrize("s,msg", [
    ("", 'time: invalid duration ""'), ("5", 'time: missing unit in duration "5"'),
    ("5x", 'time: unknown unit "x" in duration "5x"'), ("s", 'time: invalid duration "s"'),
    (".s", 'time: invalid duration ".s"'), ("-", 'time: invalid duration "-"'),
    ("3000000h", 'time: invalid duration "3000000h"'), ("1s5", 'time: missing unit in duration "1s5"'),
])
def test_parse_duration_errors(s, msg):
    with pytest.raises(GoSyntaxError) as e:
        parse_duration(s)
    assert str(e.value) == msg


@pytest.mark.parametrize("ns,s", [
    (0, "0s"), (5 * SECOND, "5s"), (10 * SECOND, "10s"), (MINUTE, "1m0s"), (5 * MINUTE, "5m0s"), (HOUR, "1h0m0s"),
    (1500 * MILLISECOND, "1.5s"), (500 * MILLISECOND, "500ms"), (1, "1ns"), (1500, "1.5µs"), (-MINUTE, "-1m0s"),
    (90 * MINUTE + 1, "1h30m0.000000001s"),
])
def test_format_duration(ns, s):
    assert format_duration(ns) == s


def _fs():
    fs = FlagSet(program="prog")
    fs.duration("poll-period", 5 * SECOND, "The interval")
    fs.int("max-pods", 5, "Max pods")
    fs.string("aws-region", "", "Your AWS region")
    fs.string("ns", "default", "namespace")
    fs.bool("v", False, "verbose")
    return fs


@pytest.mark.parametrize("argv", [
    ["-max-pods=8"], ["--max-pods=8"], ["-max-pods", "8"], ["--max-pods", "8"], ["-max-pods=0x8"], ["-max-pods", "010"],
])
def test_flag_syntaxes(argv):
    fs = _fs()
    fs.parse(argv)
    assert fs["max-pods"] == 8


def test_flag_stops_at_first_non_flag_and_double_dash():
    fs = _fs()
    fs.parse(["-max-pods=3", "pos", "-aws-region=x"])
    assert fs["max-pods"] == 3 and fs["aws-region"] == "" and fs.args == ["pos", "-aws-region=x"]
    fs = _fs()
    fs.parse(["--", "-max-pods=3"])
    assert fs["max-pods"] == 5 and fs.args == ["-max-pods=3"]
    fs = _fs()
    fs.parse(["-", "x"])  # a lone "-" is a non-flag argument
    assert fs.args == ["-", "x"]


def test_flag_last_wins_and_value_may_start_with_dash():
    fs = _fs()
    fs.parse(["-max-pods=1", "-max-pods=2", "-aws-region", "-x"])
    assert fs["max-pods"] == 2 and fs["aws-region"] == "-x"


def test_bool_flag_forms():
    fs = _fs()
    fs.parse(["-v"])
    assert fs["v"] is True
    fs = _fs()
    fs.parse(["-v=false", "rest"])
    assert fs["v"] is False and fs.args == ["rest"]
    fs = _fs()
    fs.parse(["-v", "false"])  # bool flags never consume the next argument
    assert fs["v"] is True and fs.args == ["false"]


@pytest.mark.parametrize("argv,msg", [
    (["-nope"], "flag provided but not defined: -nope"),
    (["-max-pods=abc"], 'invalid value "abc" for flag -max-pods: parse error'),
    (["-max-pods=99999999999999999999"], 'invalid value "99999999999999999999" for flag -max-pods: value out of range'),
    (["-poll-period=5"], 'invalid value "5" for flag -poll-period: parse error'),
    (["-max-pods"], "flag needs an argument: -max-pods"),
    (["---x"], "bad flag syntax: ---x"),
    (["-=x"], "bad flag syntax: -=x"),
    (["-v=maybe"], 'invalid boolean value "maybe" for -v: parse error'),
])
def test_flag_errors(argv, msg):
    with pytest.raises(FlagError) as e:
        _fs().parse(argv)
    assert str(e.value) == msg and not e.value.help


@pytest.mark.parametrize("argv", [["-h"], ["-help"], ["--help"]])
def test_help(argv):
    with pytest.raises(FlagError) as e:
        _fs().parse(argv)
    assert e.value.help


def test_usage_matches_go_print_defaults():
    assert _fs().usage() == (
        "Usage of prog:\n"
        "  -aws-region string\n    \tYour AWS region\n"
        "  -max-pods int\n    \tMax pods (default 5)\n"
        "  -ns string\n    \tnamespace (default \"default\")\n"
        "  -poll-period duration\n    \tThe interval (default 5s)\n"
        "  -v\tverbose\n"
    )


@pytest.mark.parametrize("text,want", [
    ("5", 5.0), ("0.5", 0.5), ("1e3", 1000.0), ("1_000.5", 1000.5), ("0x1p-2", 0.25), ("+2", 2.0), (".5", 0.5),
    ("Inf", float("inf")), ("-infinity", float("-inf")),
])
def test_parse_float_like_strconv(text, want):
    from kube_sqs_autoscaler_amd.utils.goflag import parse_float

    assert parse_float(text) == want


@pytest.mark.parametrize("text,err", [
    ("", "invalid syntax"), (" 1", "invalid syntax"), ("1__0", "invalid syntax"), ("0x10", "invalid syntax"),
    ("+nan", "invalid syntax"), ("1e400", "value out of range"), ("abc", "invalid syntax"), ("١", "invalid syntax"),
])
def test_parse_float_errors(text, err):
    from kube_sqs_autoscaler_amd.utils.goflag import GoRangeError, GoSyntaxError, parse_float

    with pytest.raises((GoSyntaxError, GoRangeError), match=err):
        parse_float(text)


@pytest.mark.parametrize("v,text", [(5.0, "5"), (0.5, "0.5"), (1e6, "1e+06"), (123456.0, "123456"),
                                    (1234567.0, "1.234567e+06"), (1e-4, "0.0001"), (1e-5, "1e-05"), (-3.25, "-3.25")])
def test_format_float_like_go(v, text):
    """flag.Float64's default text is strconv.FormatFloat(v, 'g', -1, 64)."""
    from kube_sqs_autoscaler_amd.utils.goflag import format_float

    assert format_float(v) == text


def test_float_flag_usage_and_errors():
    from kube_sqs_autoscaler_amd.utils.goflag import FlagError, FlagSet

    fs = FlagSet(program="p")
    fs.float64("qps", 5.0, "requests per second")
    fs.float64("zero", 0.0, "no default shown")
    assert fs.usage() == "Usage of p:\n  -qps float\n    \trequests per second (default 5)\n  -zero float\n    \tno default shown\n"
    fs.parse(["-qps", "2.5"])
    assert fs["qps"] == 2.5
    bad = FlagSet(program="p")
    bad.float64("qps", 5.0, "u")
    with pytest.raises(FlagError, match='invalid value "x" for flag -qps: parse error'):
        bad.parse(["-qps=x"])
    with pytest.raises(FlagError, match='invalid value "1e999" for flag -qps: value out of range'):
        bad.parse(["-qps=1e999"])


def test_utc_formatting_matches_the_calendar(nat):
    """rfc3339_utc / amz_date (X-Amz-Date) are formatted by arithmetic, not gmtime_r + strftime
    (glibc's tzset lock, taken per call, serialised the workers): same text as a calendar
    library over the whole int64-nanosecond range, negative times and leap days included."""
    import datetime
    import random

    rng = random.Random(7)
    cases = [0, -1, 1, 86399 * 10**9, -86400 * 10**9, 951782400 * 10**9, 4107542399 * 10**9 + 999_999_999,
             -(2**63), 2**63 - 1, 1700000000 * 10**9] + [rng.randrange(-(2**63), 2**63) for _ in range(2000)]
    epoch = datetime.datetime(1970, 1, 1)
    for ns in cases:
        dt = epoch + datetime.timedelta(microseconds=ns // 1000)  # floor, like time.Unix
        assert nat.rfc3339_utc(ns) == dt.strftime("%Y-%m-%dT%H:%M:%SZ"), ns
        assert nat.amz_date(ns) == dt.strftime("%Y%m%dT%H%M%SZ"), ns

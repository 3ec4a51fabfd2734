"""SigV4 (what aws-sdk-go did for the reference, sqs/sqs.go:36,51): published vectors + an
independent pure-Python implementation of the algorithm as a cross-check."""
import calendar
import hashlib
import hmac
import urllib.parse

import pytest

SECRET = "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY"
TS_20150830 = calendar.timegm((2015, 8, 30, 12, 36, 0)) * 10**9


def test_signing_key_published_vector(nat):
    # AWS General Reference, "Examples of how to derive a signing key" (iam, us-east-1, 20150830)
    s = nat.SigV4Signer("us-east-1", "iam")
    assert s.signing_key_hex(SECRET, "20150830") == "c4afb1cc5771d871763a393e44b703571b55cc28424d1a5e86da6ed3c154a4b9"


def test_get_vanilla_published_vector(nat):
    # aws-sig-v4-test-suite/get-vanilla
    c = nat.Credentials("AKIDEXAMPLE", SECRET, "", 0, "t")
    h, d = nat.SigV4Signer("us-east-1", "service").sign(c, TS_20150830, "GET", "/", "", [("Host", "example.amazonaws.com")], b"")
    assert d["string_to_sign"].endswith("bb579772317eb040ac9ed261061d46c1f17a8133879d6129b6e1c25292927e63")
    assert dict(h)["Authorization"] == (
        "AWS4-HMAC-SHA256 Credential=AKIDEXAMPLE/20150830/us-east-1/service/aws4_request, "
        "SignedHeaders=host;x-amz-date, Signature=5fa00fa31553b73ebf1942676e86291e8372ff2a2260956d9b8aae1d763fbf31")


def _py_sign(secret, akid, region, service, amzdate, method, path, query, headers, body, token=""):
    """Independent SigV4 from the published algorithm (no shared code with csrc/core/sigv4.cc)."""
    hdrs = {k.lower(): " ".join(v.strip().split()) for k, v in headers}
    hdrs["x-amz-date"] = amzdate
    if token:
        hdrs["x-amz-security-token"] = token
    signed = ";".join(sorted(hdrs))
    enc = lambda s: urllib.parse.quote(s, safe="-_.~")
    qs = sorted((enc(urllib.parse.unquote_plus(k)), enc(urllib.parse.unquote_plus(v)))
                for k, _, v in (p.partition("=") for p in query.split("&") if p))
    canon = "\n".join([
        # non-S3 services encode the (already escaped) path a second time
        method, urllib.parse.quote(urllib.parse.quote(path, safe="/-_.~"), safe="/-_.~"), "&".join(f"{k}={v}" for k, v in qs),
        "".join(f"{k}:{hdrs[k]}\n" for k in sorted(hdrs)), signed, hashlib.sha256(body).hexdigest()])
    date = amzdate[:8]
    scope = f"{date}/{region}/{service}/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amzdate, scope, hashlib.sha256(canon.encode()).hexdigest()])
    k = ("AWS4" + secret).encode()
    for part in (date, region, service, "aws4_request"):
        k = hmac.new(k, part.encode(), hashlib.sha256).digest()
    return hmac.new(k, sts.encode(), hashlib.sha256).hexdigest(), canon


@pytest.mark.parametrize("query,body,token,path", [
    ("", b"Action=GetQueueAttributes&AttributeName.1=ApproximateNumberOfMessages&QueueUrl=https%3A%2F%2Fsqs.us-west-2.amazonaws.com%2F1%2Fq&Version=2012-11-05", "", "/"),
    ("b=2&a=1&c=%20x", b"", "", "/"),
    ("", b'{"QueueUrl":"u"}', "FQoGZXIvYXdzEJr//////////session", "/"),
    ("Param2=value2&Param1=value1", b"", "", "/path/with space/and~tilde"),
])
def test_matches_independent_python_sigv4(nat, query, body, token, path):
    c = nat.Credentials("AKIDEXAMPLE", SECRET, token, 0, "t")
    headers = [("Host", "sqs.us-west-2.amazonaws.com"), ("Content-Type", "application/x-www-form-urlencoded; charset=utf-8")]
    ts = calendar.timegm((2024, 2, 29, 23, 59, 59)) * 10**9
    wire_path = urllib.parse.quote(path, safe="/-_.~")
    h, d = nat.SigV4Signer("us-west-2", "sqs").sign(c, ts, "POST", wire_path, query, headers, body)
    sig, canon = _py_sign(SECRET, "AKIDEXAMPLE", "us-west-2", "sqs", "20240229T235959Z", "POST", path, query, headers, body, token)
    assert d["canonical_request"] == canon
    assert d["signature"] == sig
    hd = dict(h)
    assert hd["X-Amz-Date"] == "20240229T235959Z"
    if token:
        assert hd["X-Amz-Security-Token"] == token
    # the fake server's verifier accepts it, and rejects tampering
    nat.sigv4_verify("POST", wire_path, query, h, body, "AKIDEXAMPLE", SECRET, "us-west-2", "sqs")
    with pytest.raises(nat.NativeError):
        nat.sigv4_verify("POST", wire_path, query, h, body + b"x", "AKIDEXAMPLE", SECRET, "us-west-2", "sqs")
    with pytest.raises(nat.NativeError):
        nat.sigv4_verify("POST", wire_path, query, h, body, "AKIDEXAMPLE", SECRET + "x", "us-west-2", "sqs")


def test_uri_encode(nat):
    assert nat.aws_uri_encode("a b/c~d_e.f-g+h=", False) == "a%20b%2Fc~d_e.f-g%2Bh%3D"
    assert nat.aws_uri_encode("a b/c", True) == "a%20b/c"
    assert nat.aws_uri_encode("é", False) == "%C3%A9"


def test_hash_helpers(nat):
    assert nat.sha256_hex(b"") == hashlib.sha256(b"").hexdigest()
    assert nat.hmac_sha256_hex(b"k", b"d") == hmac.new(b"k", b"d", hashlib.sha256).hexdigest()


from hypothesis import given, settings
from hypothesis import strategies as st

_hdr_names = st.sampled_from(["Host", "Content-Type", "X-Amz-Target", "x-custom", "X-Amz-Meta-A", "Accept"])
_hdr_values = st.text(alphabet=st.characters(min_codepoint=32, max_codepoint=126), max_size=20)


@settings(max_examples=200, deadline=None)
@given(headers=st.lists(st.tuples(_hdr_names, _hdr_values), max_size=5),
       body=st.binary(max_size=200), token=st.sampled_from(["", "sess/token=="]),
       query=st.sampled_from(["", "a=1&b=2", "z=%20x&a=b"]), path=st.sampled_from(["/", "/123/queue", "/a b"]),
       ts=st.integers(1_500_000_000, 2_000_000_000))
def test_prepared_signing_equals_generic(nat, headers, body, token, query, path, ts):
    """The per-queue fast path (prepare once, sign the date) == the generic signer, byte for byte."""
    c = nat.Credentials("AKIDEXAMPLE", SECRET, token, 0, "t")
    s = nat.SigV4Signer("us-west-2", "sqs")
    hs = [("Host", "sqs.us-west-2.amazonaws.com")] + list(headers)
    h1, d1 = s.sign(c, ts * 10**9, "POST", path, query, hs, body)
    h2, d2 = s.sign_prepared(c, ts * 10**9, "POST", path, query, hs, body)
    assert d1["canonical_request"] == d2["canonical_request"]
    assert d1["signature"] == d2["signature"] and dict(h1)["Authorization"] == dict(h2)["Authorization"]
    # the allocation-free path taken per poll (no debug capture; in place without a token)
    h3 = s.sign_prepared_headers(c, ts * 10**9, "POST", path, query, hs, body)
    assert h3 == h2

"""session.Must(session.NewSession()) start-up validation (/root/reference/sqs/sqs.go:36; the panic
happens before ``Starting kube-sqs-autoscaler``, main.go:112-114). sqs/session.py."""
import os
import subprocess
import sys

import pytest
import yaml

from kube_sqs_autoscaler_amd.sqs.session import SessionError, custom_ca_bundle, go_parse_bool, validate_session

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def home(tmp_path):
    """An empty HOME (no ~/.aws files) and env keys, so only what a test adds is checked."""
    return {"HOME": str(tmp_path), "AWS_ACCESS_KEY_ID": "AKID", "AWS_SECRET_ACCESS_KEY": "S"}


def _cert_pem(nat) -> str:
    s = nat.FakeSqsServer()
    s.start("127.0.0.1", 0, True)
    try:
        return s.cert_pem
    finally:
        s.stop()


def test_valid_and_empty_environments_pass(home, tmp_path):
    validate_session(home)
    validate_session({"HOME": str(tmp_path)})  # nothing configured: lazily "NoCredentialProviders" later
    (tmp_path / ".aws").mkdir()
    (tmp_path / ".aws" / "credentials").write_text("[default]\naws_access_key_id = A\naws_secret_access_key = B\n")
    validate_session({"HOME": str(tmp_path), "AWS_STS_REGIONAL_ENDPOINTS": "Regional"})  # case-insensitive
    validate_session({**home, "AWS_SHARED_CREDENTIALS_FILE": str(tmp_path / "missing")})  # unreadable: skipped


@pytest.mark.parametrize("key,val,msg", [
    ("AWS_STS_REGIONAL_ENDPOINTS", "global",
     "failed to load environment config, failed to load, AWS_STS_REGIONAL_ENDPOINTS from env config, "
     "unable to resolve the value of STSRegionalEndpoint for global"),
    ("AWS_S3_US_EAST_1_REGIONAL_ENDPOINT", "x",
     "failed to load environment config, failed to load, AWS_S3_US_EAST_1_REGIONAL_ENDPOINT from env config, "
     "unable to resolve the value of S3UsEast1RegionalEndpoint for x"),
    ("AWS_S3_USE_ARN_REGION", "yes",
     "failed to load environment config, invalid value for environment variable, AWS_S3_USE_ARN_REGION=yes, "
     "need true or false"),
])
def test_invalid_env_values(home, key, val, msg):
    with pytest.raises(SessionError) as e:
        validate_session({**home, key: val})
    assert str(e.value) == msg


def test_ca_bundle(home, tmp_path, nat):
    with pytest.raises(SessionError) as e:
        validate_session({**home, "AWS_CA_BUNDLE": str(tmp_path / "nope.pem")})
    assert str(e.value) == ("LoadCustomCABundleError: failed to open custom CA bundle PEM file\n"
                            f"caused by: open {tmp_path / 'nope.pem'}: no such file or directory")
    junk = tmp_path / "junk.pem"
    junk.write_text("-----BEGIN CERTIFICATE-----\nnot base64\n-----END CERTIFICATE-----\n")
    with pytest.raises(SessionError, match="^LoadCustomCABundleError: failed to load custom CA bundle PEM file$"):
        validate_session({**home, "AWS_CA_BUNDLE": str(junk)})
    with pytest.raises(SessionError, match="failed to read custom CA bundle PEM file\ncaused by: read .*: is a directory"):
        validate_session({**home, "AWS_CA_BUNDLE": str(tmp_path)})
    good = tmp_path / "ca.pem"
    good.write_text("comment lines are ignored\n" + _cert_pem(nat))
    validate_session({**home, "AWS_CA_BUNDLE": str(good)})


def test_unparsable_shared_files(home, tmp_path):
    """Only a section header without its ']' fails the session (the SDK's lexer cannot get past
    it either); the config file is only read with AWS_SDK_LOAD_CONFIG."""
    bad = tmp_path / "bad"
    bad.write_text("[default\naws_access_key_id = AKID\n")
    with pytest.raises(SessionError) as e:
        validate_session({**home, "AWS_SHARED_CREDENTIALS_FILE": str(bad)})
    assert str(e.value).startswith(f"SharedConfigLoadError: failed to load config file, {bad}\ncaused by: ")
    assert "section header without a closing ']'" in str(e.value)
    # the config file is only read with AWS_SDK_LOAD_CONFIG (Go ParseBool: "yes" is false)
    env = {**home, "AWS_CONFIG_FILE": str(bad)}
    validate_session(env)
    validate_session({**env, "AWS_SDK_LOAD_CONFIG": "yes"})
    with pytest.raises(SessionError, match="SharedConfigLoadError"):
        validate_session({**env, "AWS_SDK_LOAD_CONFIG": "1"})


@pytest.mark.parametrize("text,warned", [
    ("aws_access_key_id = outside any section\n[default]\naws_access_key_id = A\naws_secret_access_key = S\n",
     "key outside any [section]"),
    ("[default]\nnot an assignment\naws_access_key_id = A\naws_secret_access_key = S\n", "not a key = value line"),
    ("# comment\n; comment\n\n[default]\naws_access_key_id = A ; inline text stays in the value\n"
     "aws_secret_access_key: S\n[default]\ns3 =\n  max_concurrent_requests = 10\n", None),
])
def test_shared_files_the_sdk_may_accept_are_loaded_with_warnings(home, tmp_path, text, warned):
    """Constructs the SDK's ini parser may well accept (parity unpinned: no SDK here) do not
    crash-loop the pod: the unusable lines are skipped and reported as warnings, and the rest of
    the file -- here the default profile's keys -- is used."""
    from kube_sqs_autoscaler_amd.sqs import ini

    f = tmp_path / "credentials"
    f.write_text(text)
    warnings = validate_session({**home, "AWS_SHARED_CREDENTIALS_FILE": str(f)})
    if warned:
        assert len(warnings) == 1 and warned in warnings[0] and str(f) in warnings[0]
    else:
        assert warnings == []
    parsed = ini.read(str(f))
    d = dict(parsed.items("default"))
    assert d["aws_access_key_id"].startswith("A") and d["aws_secret_access_key"] == "S"
    if warned is None:
        assert d["aws_access_key_id"] == "A ; inline text stays in the value"
        assert d["s3"] == "\nmax_concurrent_requests = 10"


def test_profile_checks_with_load_config(home, tmp_path):
    cfg = tmp_path / "config"
    env = {"HOME": str(tmp_path), "AWS_CONFIG_FILE": str(cfg), "AWS_SDK_LOAD_CONFIG": "true"}
    cfg.write_text("[default]\nsts_regional_endpoints = sometimes\n")
    with pytest.raises(SessionError) as e:
        validate_session(env)
    assert str(e.value) == f"failed to load sts_regional_endpoints from shared config, {cfg}, sometimes"
    cfg.write_text("[profile p]\nrole_arn = arn:aws:iam::1:role/r\nsource_profile = ghost\n")
    with pytest.raises(SessionError, match="failed to load assume role for arn:aws:iam::1:role/r, source profile ghost "
                                           "has no shared credentials"):
        validate_session({**env, "AWS_PROFILE": "p"})
    cfg.write_text("[profile p]\nsource_profile = base\n[profile base]\naws_access_key_id = A\naws_secret_access_key = B\n")
    with pytest.raises(SessionError, match="CredentialRequiresARNError: credential type source_profile requires role_arn"):
        validate_session({**env, "AWS_PROFILE": "p"})
    cfg.write_text("[default]\nrole_arn = arn:aws:iam::1:role/r\ncredential_source = Lambda\n")
    with pytest.raises(SessionError, match="credential source values must be EcsContainer, Ec2InstanceMetadata, or Environment"):
        validate_session(env)
    cfg.write_text("[default]\nrole_arn = arn:aws:iam::1:role/r\ncredential_source = EcsContainer\n")
    with pytest.raises(SessionError, match="'AWS_CONTAINER_CREDENTIALS_RELATIVE_URI' was not set"):
        validate_session(env)
    validate_session({**env, "AWS_CONTAINER_CREDENTIALS_RELATIVE_URI": "/v2/creds"})
    cfg.write_text("[default]\nrole_arn = arn:aws:iam::1:role/r\nsource_profile = base\nmfa_serial = arn:mfa\n"
                   "[profile base]\naws_access_key_id = A\naws_secret_access_key = B\n")
    with pytest.raises(SessionError, match="^AssumeRoleTokenProviderNotSetError"):
        validate_session(env)
    # a valid assume-role chain, and a self-linked profile
    cfg.write_text("[default]\nrole_arn = arn:aws:iam::1:role/r\nsource_profile = default\n"
                   "aws_access_key_id = A\naws_secret_access_key = B\n")
    validate_session(env)
    # environment keys win over the profile's credential wiring
    cfg.write_text("[default]\nrole_arn = arn:aws:iam::1:role/r\ncredential_source = Lambda\n")
    validate_session({**env, "AWS_ACCESS_KEY_ID": "A", "AWS_SECRET_ACCESS_KEY": "B"})


def test_web_identity_needs_role_arn(tmp_path):
    env = {"HOME": str(tmp_path), "AWS_WEB_IDENTITY_TOKEN_FILE": str(tmp_path / "token")}
    with pytest.raises(SessionError, match="^WebIdentityErr: role ARN is not set$"):
        validate_session(env)
    validate_session({**env, "AWS_ROLE_ARN": "arn:aws:iam::1:role/irsa"})  # the token file is read lazily


def test_profile_ca_bundle(tmp_path, nat):
    pem = tmp_path / "ca.pem"
    pem.write_text(_cert_pem(nat))
    cfg = tmp_path / "config"
    cfg.write_text(f"[default]\nca_bundle = {pem}\n")
    env = {"HOME": str(tmp_path), "AWS_CONFIG_FILE": str(cfg), "AWS_SDK_LOAD_CONFIG": "1"}
    assert custom_ca_bundle(env) == str(pem)
    assert custom_ca_bundle({**env, "AWS_CA_BUNDLE": "/env.pem"}) == "/env.pem"
    assert custom_ca_bundle({**env, "AWS_SDK_LOAD_CONFIG": "0"}) == ""
    validate_session(env)
    cfg.write_text(f"[default]\nca_bundle = {tmp_path / 'gone.pem'}\n")
    with pytest.raises(SessionError, match="failed to open custom CA bundle PEM file"):
        validate_session(env)


def test_go_parse_bool():
    assert all(go_parse_bool(v) for v in ("1", "t", "T", "TRUE", "true", "True"))
    assert not any(go_parse_bool(v) for v in ("", "yes", "on", "tRUE", "0", "false", None))


# ---- the CLI: panic + exit 2 before the start-up line ----------------------------------------


def _kubeconfig(tmp_path) -> str:
    kc = tmp_path / "kubeconfig"
    kc.write_text(yaml.safe_dump({
        "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": "http://127.0.0.1:9"}}],
        "users": [{"name": "u", "user": {"token": "t"}}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
    return str(kc)


def _run(tmp_path, extra):
    e = dict(os.environ)
    for k in list(e):
        if k.startswith("AWS_"):
            del e[k]
    e.update({"HOME": str(tmp_path), "KUBE_CONFIG_PATH": _kubeconfig(tmp_path), **extra})
    return subprocess.run([sys.executable, "-m", "kube_sqs_autoscaler_amd", "--sqs-queue-url=http://127.0.0.1:9/1/q",
                           "--kubernetes-deployment=w", "--aws-region=us-east-1", "--max-pods=8"], cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=60)


def test_cli_panics_on_bad_session(tmp_path):
    bad = tmp_path / "credentials"
    bad.write_text("[default\nnot an ini file\n")
    cases = [
        ({"AWS_SHARED_CREDENTIALS_FILE": str(bad)}, "panic: SharedConfigLoadError: failed to load config file, "),
        ({"AWS_CONFIG_FILE": str(bad), "AWS_SDK_LOAD_CONFIG": "1"}, "panic: SharedConfigLoadError: failed to load config file, "),
        ({"AWS_CA_BUNDLE": str(tmp_path / "missing.pem")},
         "panic: LoadCustomCABundleError: failed to open custom CA bundle PEM file\ncaused by: open "),
        ({"AWS_STS_REGIONAL_ENDPOINTS": "global"}, "panic: failed to load environment config, failed to load, "
                                                   "AWS_STS_REGIONAL_ENDPOINTS from env config"),
    ]
    for env, want in cases:
        r = _run(tmp_path, env)
        assert r.returncode == 2, (env, r.stderr)
        assert r.stderr.startswith(want), (env, r.stderr)
        assert "Starting kube-sqs-autoscaler" not in r.stderr


def test_cli_kube_config_panic_comes_first(tmp_path):
    """NewPodAutoScaler runs before NewSqsClient (main.go:101,112): a broken kube config wins."""
    e = dict(os.environ)
    e.pop("KUBE_CONFIG_PATH", None)
    e.update({"HOME": str(tmp_path), "KUBERNETES_SERVICE_HOST": "", "AWS_STS_REGIONAL_ENDPOINTS": "global"})
    r = subprocess.run([sys.executable, "-m", "kube_sqs_autoscaler_amd"], cwd=ROOT, env=e, capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 2 and "panic: Failed to configure incluster or local config" in r.stderr


def test_cli_valid_session_starts(tmp_path, nat):
    """A valid configuration is unaffected: the loop starts and polls."""
    from kube_sqs_autoscaler_amd.cli import main

    sqs = nat.FakeSqsServer()
    sqs.start()
    kube = nat.FakeKubeServer()
    kube.start()
    try:
        kube.add_deployment("default", "w", 1)
        url = sqs.url + "/1/q"
        sqs.set_attributes(url, {"ApproximateNumberOfMessages": "0", "ApproximateNumberOfMessagesDelayed": "0",
                                 "ApproximateNumberOfMessagesNotVisible": "0"})
        kc = tmp_path / "kc"
        kc.write_text(yaml.safe_dump({
            "current-context": "t", "clusters": [{"name": "c", "cluster": {"server": kube.url}}],
            "users": [{"name": "u", "user": {"token": "t"}}], "contexts": [{"name": "t", "context": {"cluster": "c", "user": "u"}}]}))
        cfg = tmp_path / "config"
        cfg.write_text("[default]\nsts_regional_endpoints = regional\nregion = us-east-1\n")
        env = {"HOME": str(tmp_path), "KUBE_CONFIG_PATH": str(kc), "AWS_ACCESS_KEY_ID": "A", "AWS_SECRET_ACCESS_KEY": "B",
               "AWS_CONFIG_FILE": str(cfg), "AWS_SDK_LOAD_CONFIG": "1", "AWS_STS_REGIONAL_ENDPOINTS": "legacy"}
        assert main([f"--sqs-queue-url={url}", "--kubernetes-deployment=w", f"--sqs-endpoint={sqs.url}", "--aws-region=us-east-1",
                     "--poll-period=1ms", "--max-pods=8"], environ=env, max_iterations=3) == 0
        assert sqs.requests() == 3
    finally:
        sqs.stop()
        kube.stop()


def test_shared_file_reader_fails_only_on_an_unclosed_section_header():
    """Property: whatever the lines, the reader raises only when a line starts a section header
    it never closes; every other input parses (unusable lines become warnings)."""
    from hypothesis import given, settings
    from hypothesis import strategies as st

    from kube_sqs_autoscaler_amd.sqs import ini

    no_breaks = st.characters(blacklist_categories=("Cs",),
                              blacklist_characters="\r\n\x0b\x0c\x1c\x1d\x1e\x85\u2028\u2029")
    line = st.one_of(st.text(alphabet=no_breaks, max_size=30),
                     st.sampled_from(["[default]", "[profile x]", "key = value", "  continued", "# c", "; c", "=v",
                                      ":v", "[", "[open"]))

    @settings(max_examples=300, deadline=None)
    @given(st.lists(line, max_size=12))
    def check(lines):
        text = "\n".join(lines)
        unclosed = any(l.strip().startswith("[") and "]" not in l.strip() for l in lines)
        try:
            f = ini.parse(text, "f")
        except ini.IniError:
            assert unclosed, lines
            return
        assert not unclosed or all(  # an unclosed header inside a continuation is just text
            l[:1] in (" ", "\t") for l in lines if l.strip().startswith("[") and "]" not in l.strip()), lines
        for sec in f.sections():
            for k, _ in f.items(sec):
                assert k == k.lower()

    check()


def test_indented_keys_and_headers_are_keys_and_headers():
    """a line continues the previous value only when indented deeper than that key's
    line (configparser's rule), so a file whose keys (or headers) are indented alike parses key by
    key; the SDK's nested ``s3 =`` block still folds into its key."""
    from kube_sqs_autoscaler_amd.sqs import ini

    f = ini.parse("[default]\n  aws_access_key_id = A\n  aws_secret_access_key = B\n"
                  "  [profile x]\n  region = eu-west-1\n  s3 =\n    max_concurrent_requests = 20\n"
                  "    addressing_style = path\n  output = json\n", "f")
    assert dict(f.items("default")) == {"aws_access_key_id": "A", "aws_secret_access_key": "B"}
    assert dict(f.items("profile x")) == {"region": "eu-west-1", "output": "json",
                                          "s3": "\nmax_concurrent_requests = 20\naddressing_style = path"}
    # unindented keys: an indented line is a continuation, as before
    g = ini.parse("[default]\nkey = a\n  b\nother = c\n", "g")
    assert dict(g.items("default")) == {"key": "a\nb", "other": "c"}


def test_uniform_indent_reads_like_no_indent():
    """Property: indenting every header and key line by the same amount changes nothing -- the
    same sections, keys and values as the unindented file (continuations stay deeper)."""
    from hypothesis import given, settings
    from hypothesis import strategies as st

    from kube_sqs_autoscaler_amd.sqs import ini

    word = st.text(alphabet="abcdefghijklmnopqrstuvwxyz_0123456789", min_size=1, max_size=8)
    entry = st.tuples(word, word, st.lists(word, max_size=2))  # key, value, continuation lines
    sections = st.lists(st.tuples(word, st.lists(entry, max_size=4)), min_size=1, max_size=3)

    def render(secs, pad: str) -> str:
        out = []
        for name, entries in secs:
            out.append(f"{pad}[{name}]")
            for key, value, more in entries:
                out.append(f"{pad}{key} = {value}")
                out.extend(f"{pad}    {m}" for m in more)
        return "\n".join(out) + "\n"

    @settings(max_examples=200, deadline=None)
    @given(sections, st.sampled_from(["  ", "\t", "    "]))
    def check(secs, pad):
        flat, indented = ini.parse(render(secs, ""), "f"), ini.parse(render(secs, pad), "g")
        assert flat.sections() == indented.sections()
        for s in flat.sections():
            assert flat.items(s) == indented.items(s)

    check()


def test_indented_credentials_file_feeds_the_chain(tmp_path):
    from kube_sqs_autoscaler_amd.sqs.credentials import SharedFileProvider

    p = tmp_path / "credentials"
    p.write_text("[default]\n  aws_access_key_id = AKIDINDENT\n  aws_secret_access_key = SECRETINDENT\n")
    c = SharedFileProvider({"AWS_SHARED_CREDENTIALS_FILE": str(p), "HOME": str(tmp_path)}).fetch()
    assert c.access_key_id == "AKIDINDENT" and c.secret_access_key == "SECRETINDENT"

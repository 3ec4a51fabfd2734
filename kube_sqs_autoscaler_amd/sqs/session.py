"""Start-up validation of the AWS session: what ``session.Must(session.NewSession())`` checks.

The reference builds its SQS client with ``sqs.New(session.Must(session.NewSession()), ...)``
(/root/reference/sqs/sqs.go:36), right after the kube client (main.go:101,112) and before
``Starting kube-sqs-autoscaler`` (main.go:114). ``NewSession`` does no network I/O and fetches
no credentials (those resolve lazily on the first call, sqs/credentials.py), but it does read
and check its configuration, and ``session.Must`` panics on any error: the process prints
``panic: <error>`` and exits 2 before the loop starts, so a misconfigured pod crash-loops
instead of logging one error per poll. aws-sdk-go v1.35.35's checks (go.mod:6), in its order:

1. the environment (``loadEnvConfig``): ``AWS_STS_REGIONAL_ENDPOINTS`` and
   ``AWS_S3_US_EAST_1_REGIONAL_ENDPOINT`` must be ``legacy`` or ``regional``,
   ``AWS_S3_USE_ARN_REGION`` ``true`` or ``false`` (any case);
2. ``AWS_CA_BUNDLE`` must open;
3. the shared files (the credentials file; with ``AWS_SDK_LOAD_CONFIG`` the config file first):
   a file that cannot be read is skipped, one that cannot be parsed is an error; with
   ``AWS_SDK_LOAD_CONFIG`` the profile's ``sts_regional_endpoints`` must be valid, and an
   assume-role profile's ``source_profile`` must exist and carry credentials;
4. credentials: web identity from the environment needs ``AWS_ROLE_ARN``; a
   ``credential_source`` must be ``EcsContainer`` (which needs
   ``AWS_CONTAINER_CREDENTIALS_RELATIVE_URI``), ``Ec2InstanceMetadata`` or ``Environment``; an
   assume-role profile with ``mfa_serial`` needs a token provider the reference never sets;
5. the CA bundle (``AWS_CA_BUNDLE``, else the profile's ``ca_bundle`` with
   ``AWS_SDK_LOAD_CONFIG``) must hold at least one certificate.

Error texts are the SDK's (``awserr``: ``Code: message`` plus ``\\ncaused by: <cause>``). The
shared files are read by :mod:`.ini`, which fails only on a section header without its ``]``
and skips (with a warning the CLI logs) lines it cannot use -- which malformed files the SDK's
own ini parser rejects is parity unpinned, and crash-looping on a file the reference loads
would be the worse error. The cause of a parse error is this parser's wording; the code,
message and file name are the SDK's.
"""
from __future__ import annotations

import os
import ssl
from typing import Dict, List, Mapping, Optional, Tuple

from . import ini


class SessionError(Exception):
    """``session.NewSession`` failed; the reference panics with this text (exit 2)."""


def go_parse_bool(v: Optional[str]) -> bool:
    """Go's ``strconv.ParseBool`` truth (``AWS_SDK_LOAD_CONFIG``); anything unparsable is false."""
    return (v or "") in ("1", "t", "T", "TRUE", "true", "True")


def load_config_enabled(environ: Mapping[str, str]) -> bool:
    return go_parse_bool(environ.get("AWS_SDK_LOAD_CONFIG"))


def session_profile(environ: Mapping[str, str]) -> str:
    """``AWS_PROFILE``; ``AWS_DEFAULT_PROFILE`` only with ``AWS_SDK_LOAD_CONFIG`` (envConfigLoad)."""
    p = environ.get("AWS_PROFILE", "")
    if not p and load_config_enabled(environ):
        p = environ.get("AWS_DEFAULT_PROFILE", "")
    return p or "default"


def shared_files(environ: Mapping[str, str]) -> List[str]:
    """The files ``NewSession`` loads, in load order (later files win)."""
    home = environ.get("HOME") or os.path.expanduser("~")
    creds = environ.get("AWS_SHARED_CREDENTIALS_FILE") or os.path.join(home, ".aws", "credentials")
    if not load_config_enabled(environ):
        return [creds]
    return [environ.get("AWS_CONFIG_FILE") or os.path.join(home, ".aws", "config"), creds]


def _go_errno_text(e: OSError) -> str:
    # Go's syscall.Errno strings are strerror(3) in lower case ("no such file or directory")
    msg = e.strerror or str(e)
    return msg[:1].lower() + msg[1:]


def _read_ini(path: str) -> Optional[ini.IniFile]:
    """A shared file, or None when it cannot be read (the SDK skips such files)."""
    try:
        return ini.read(path)
    except ini.IniError as e:
        raise SessionError(f"SharedConfigLoadError: failed to load config file, {path}\ncaused by: {e}")


_REGIONAL = ("legacy", "regional")


def _check_env(environ: Mapping[str, str]) -> None:
    pre = "failed to load environment config, "
    for key, what in (("AWS_STS_REGIONAL_ENDPOINTS", "STSRegionalEndpoint"),
                      ("AWS_S3_US_EAST_1_REGIONAL_ENDPOINT", "S3UsEast1RegionalEndpoint")):
        v = environ.get(key, "")
        if v and v.lower() not in _REGIONAL:
            raise SessionError(f"{pre}failed to load, {key} from env config, unable to resolve the value of {what} for {v}")
    v = environ.get("AWS_S3_USE_ARN_REGION", "")
    if v and v.lower() not in ("true", "false"):
        raise SessionError(f"{pre}invalid value for environment variable, AWS_S3_USE_ARN_REGION={v}, need true or false")


def _open_ca(path: str) -> bytes:
    try:
        if os.path.isdir(path):  # Go opens a directory; reading it fails
            raise SessionError("LoadCustomCABundleError: failed to read custom CA bundle PEM file\n"
                               f"caused by: read {path}: is a directory")
        with open(path, "rb") as f:
            return f.read()
    except OSError as e:
        raise SessionError(f"LoadCustomCABundleError: failed to open custom CA bundle PEM file\n"
                           f"caused by: open {path}: {_go_errno_text(e)}")


def _pem_has_certificate(data: bytes) -> bool:
    """``x509.CertPool.AppendCertsFromPEM``: true when at least one CERTIFICATE block parses."""
    text = data.decode("latin-1")
    begin, end = "-----BEGIN CERTIFICATE-----", "-----END CERTIFICATE-----"
    i = 0
    while True:
        a = text.find(begin, i)
        if a < 0:
            return False
        b = text.find(end, a)
        if b < 0:
            return False
        block = text[a:b + len(end)]
        i = b + len(end)
        try:
            ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT).load_verify_locations(cadata=block)
            return True
        except (ssl.SSLError, ValueError):
            continue


def _profile(name: str, files: List[Tuple[str, ini.IniFile]], ex_opts: bool,
             seen: set) -> Optional[Dict[str, str]]:
    """``sharedConfig.setFromIniFiles``: the profile's options merged over the files (None if no
    file has it), with the assume-role checks. Raises SessionError."""
    cfg: Dict[str, str] = {}
    found = False
    for path, cp in files:
        sec = name if cp.has_section(name) else (f"profile {name}" if cp.has_section(f"profile {name}") else None)
        if sec is None:
            continue
        found = True
        d = {k: v.strip() for k, v in cp.items(sec)}
        if d.get("aws_access_key_id") and d.get("aws_secret_access_key"):
            cfg["__creds"] = "1"
        if ex_opts:
            for k in ("role_arn", "external_id", "mfa_serial", "role_session_name", "source_profile", "credential_source",
                      "region", "ca_bundle"):
                if d.get(k):
                    cfg[k] = d[k]
            v = d.get("sts_regional_endpoints", "")
            if v and v.lower() not in _REGIONAL:
                raise SessionError(f"failed to load sts_regional_endpoints from shared config, {path}, {v}")
        for k in ("credential_process", "web_identity_token_file"):
            if d.get(k):
                cfg[k] = d[k]
    if not found:
        return None
    if name in seen:  # a self-linked profile only provides credentials
        for k in ("role_arn", "source_profile", "credential_source", "external_id", "mfa_serial", "role_session_name"):
            cfg.pop(k, None)
    else:
        for k in ("source_profile", "credential_source", "web_identity_token_file"):
            if cfg.get(k) and not cfg.get("role_arn"):
                raise SessionError(f"CredentialRequiresARNError: credential type {k} requires role_arn, profile {name}")
    seen.add(name)
    if sum(bool(cfg.get(k)) for k in ("source_profile", "credential_source", "credential_process",
                                      "web_identity_token_file")) > 1:
        raise SessionError("SharedConfigErr: only one credential type may be specified per profile: source profile, "
                           "credential source, credential process, web identity token, or sso")
    if cfg.get("source_profile"):
        for k in ("__creds", "credential_process", "web_identity_token_file", "credential_source"):
            cfg.pop(k, None)
        src = _profile(cfg["source_profile"], files, ex_opts, seen)
        if src is None or not any(src.get(k) for k in ("source_profile", "credential_source", "credential_process",
                                                         "web_identity_token_file", "__creds")):
            raise SessionError(f"SharedConfigErr: failed to load assume role for {cfg.get('role_arn', '')}, "
                               f"source profile {cfg['source_profile']} has no shared credentials")
        cfg["__source"] = src  # type: ignore[assignment]
    return cfg


def _check_profile_creds(cfg: Dict, environ: Mapping[str, str]) -> None:
    """``resolveCredsFromProfile``: the errors raised while wiring (not fetching) credentials."""
    if cfg.get("__source"):
        _check_profile_creds(cfg["__source"], environ)
    elif cfg.get("__creds") or cfg.get("credential_process"):
        pass
    elif cfg.get("credential_source"):
        cs = cfg["credential_source"]
        if cs == "EcsContainer":
            if not environ.get("AWS_CONTAINER_CREDENTIALS_RELATIVE_URI"):
                raise SessionError("SharedConfigErr: EcsContainer was specified as the credential_source, but "
                                   "'AWS_CONTAINER_CREDENTIALS_RELATIVE_URI' was not set")
        elif cs not in ("Ec2InstanceMetadata", "Environment"):
            raise SessionError("SharedConfigErr: credential source values must be EcsContainer, Ec2InstanceMetadata, "
                               "or Environment")
    elif cfg.get("web_identity_token_file"):
        if not cfg.get("role_arn"):
            raise SessionError("WebIdentityErr: role ARN is not set")
        return
    if cfg.get("role_arn") and cfg.get("mfa_serial"):
        raise SessionError("AssumeRoleTokenProviderNotSetError: assume role with MFA enabled, but "
                           "AssumeRoleTokenProvider session option not set.")


def custom_ca_bundle(environ: Mapping[str, str]) -> str:
    """The CA bundle path the session's HTTP client trusts ("" for the system roots):
    ``AWS_CA_BUNDLE``, else (with ``AWS_SDK_LOAD_CONFIG``) the profile's ``ca_bundle``."""
    if environ.get("AWS_CA_BUNDLE"):
        return environ["AWS_CA_BUNDLE"]
    if not load_config_enabled(environ):
        return ""
    files = []
    for path in shared_files(environ):
        try:
            cp = _read_ini(path)
        except SessionError:
            return ""
        if cp is not None:
            files.append((path, cp))
    try:
        prof = _profile(session_profile(environ), files, True, set())
    except SessionError:
        return ""
    return (prof or {}).get("ca_bundle", "")


def validate_session(environ: Mapping[str, str]) -> List[str]:
    """Raises :class:`SessionError` where ``session.NewSession()`` would fail; returns the
    shared files' skipped-line warnings (:mod:`.ini`) for the caller to log."""
    _check_env(environ)
    env_ca = environ.get("AWS_CA_BUNDLE", "")
    ca_data = _open_ca(env_ca) if env_ca else None
    ex_opts = load_config_enabled(environ)
    files = []
    warnings: List[str] = []
    for path in shared_files(environ):
        cp = _read_ini(path)
        if cp is not None:
            files.append((path, cp))
            warnings += cp.warnings
    prof: Optional[Dict] = None
    try:
        prof = _profile(session_profile(environ), files, ex_opts, set())
    except SessionError as e:
        # with AWS_PROFILE set, a source collision drops to the environment's credentials
        if not (environ.get("AWS_PROFILE") and "only one credential type" in str(e)):
            raise
    prof = prof or {}
    env_keys = bool((environ.get("AWS_ACCESS_KEY_ID") or environ.get("AWS_ACCESS_KEY")) and
                    (environ.get("AWS_SECRET_ACCESS_KEY") or environ.get("AWS_SECRET_KEY")))
    if not env_keys:
        if environ.get("AWS_WEB_IDENTITY_TOKEN_FILE"):
            if not environ.get("AWS_ROLE_ARN"):
                raise SessionError("WebIdentityErr: role ARN is not set")
        else:
            _check_profile_creds(prof, environ)
    if ca_data is None and prof.get("ca_bundle"):
        ca_data = _open_ca(prof["ca_bundle"])
    if ca_data is not None and not _pem_has_certificate(ca_data):
        raise SessionError("LoadCustomCABundleError: failed to load custom CA bundle PEM file")
    return warnings

"""AWS credential chain (what ``session.NewSession()`` resolves for the reference).

The reference builds its SQS client with ``sqs.New(session.Must(session.NewSession()), ...)``
(/root/reference/sqs/sqs.go:36) and never names a credential source, so it gets aws-sdk-go
v1.35.35's resolution order (go.mod:6):

1. static keys from the environment (``AWS_ACCESS_KEY_ID``/``AWS_ACCESS_KEY`` +
   ``AWS_SECRET_ACCESS_KEY``/``AWS_SECRET_KEY`` [+ ``AWS_SESSION_TOKEN``]);
2. web identity (IRSA): ``AWS_WEB_IDENTITY_TOKEN_FILE`` + ``AWS_ROLE_ARN`` ->
   STS ``AssumeRoleWithWebIdentity``;
3. the shared credentials file (``AWS_SHARED_CREDENTIALS_FILE`` or ``~/.aws/credentials``,
   profile ``AWS_PROFILE`` / ``AWS_DEFAULT_PROFILE`` / ``default``), including
   ``credential_process``; with ``AWS_SDK_LOAD_CONFIG`` also ``~/.aws/config``
   (``AWS_CONFIG_FILE``) profiles, and ``role_arn`` + ``source_profile`` /
   ``credential_source`` profiles resolve through a SigV4-signed STS ``AssumeRole`` (chains
   allowed);
4. remote: ECS task role (``AWS_CONTAINER_CREDENTIALS_RELATIVE_URI`` /
   ``AWS_CONTAINER_CREDENTIALS_FULL_URI`` + ``AWS_CONTAINER_AUTHORIZATION_TOKEN``), otherwise
   the EC2 instance role through IMDSv2 (token PUT, falling back to IMDSv1). A plain-http
   ``FULL_URI`` must name a loopback host, as in the SDK; as an extension (what later SDKs
   added for EKS Pod Identity) the Pod Identity Agent's addresses 169.254.170.23 /
   fd00:ec2::23 are accepted too, and ``AWS_CONTAINER_AUTHORIZATION_TOKEN_FILE`` (re-read on
   every fetch: the agent's token rotates) takes precedence over the inline token.

Resolution is lazy: nothing is fetched until the first poll (like the SDK), and the native
``CachedCredentials`` (csrc/core/sigv4.h) only calls :meth:`ChainProvider.retrieve` again
when the cached keys are within 5 minutes of expiry or after an ``ExpiredToken`` response.
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import threading
import urllib.error
import urllib.parse
import urllib.request
from datetime import datetime, timezone
from typing import Callable, Dict, List, Mapping, Optional, Tuple

from ..ops import native
from . import ini
from ..utils import proxy

ECS_HOST = "http://169.254.170.2"
IMDS_HOST = "http://169.254.169.254"


class CredentialsError(RuntimeError):
    pass


def parse_expiration(s: str) -> int:
    """ISO-8601 (``2024-05-01T12:00:00Z`` or with offset / fraction) -> unix nanoseconds."""
    s = s.strip()
    if s.endswith("Z") or s.endswith("z"):
        s = s[:-1] + "+00:00"
    # Python 3.10's fromisoformat wants exactly 3 or 6 fractional digits
    m = re.match(r"^(.*T\d\d:\d\d:\d\d)(?:\.(\d+))?(.*)$", s)
    if m:
        frac = (m.group(2) or "")[:6]
        s = m.group(1) + ("." + frac.ljust(6, "0") if frac else "") + m.group(3)
    dt = datetime.fromisoformat(s)
    if dt.tzinfo is None:
        dt = dt.replace(tzinfo=timezone.utc)
    return int(dt.timestamp()) * 1_000_000_000 + dt.microsecond * 1000


Fetch = Callable[[str, str, Dict[str, str], bytes, float], Tuple[int, bytes]]


def urllib_fetch(method: str, url: str, headers: Dict[str, str], body: bytes, timeout: float) -> Tuple[int, bytes]:
    req = urllib.request.Request(url, data=body if body else None, method=method, headers=headers)
    # Go's proxy rules (NO_PROXY CIDRs, loopback), not urllib's own environment handling
    p = proxy.select(url)
    opener = urllib.request.build_opener(urllib.request.ProxyHandler({urllib.parse.urlsplit(url).scheme: p} if p else {}))
    try:
        with opener.open(req, timeout=timeout) as r:
            return r.status, r.read()
    except urllib.error.HTTPError as e:
        # closed here, on the calling thread: it may be a control-loop worker on a file table
        # of its own (Supervisor), where a socket must not be left for another thread to close
        try:
            return e.code, e.read()
        finally:
            e.close()


def _make(akid: str, secret: str, token: str, expires_ns: int, name: str):
    return native().Credentials(akid, secret, token, expires_ns, name)


class _Provider:
    name = "provider"

    def fetch(self):  # -> native Credentials
        raise NotImplementedError


class EnvProvider(_Provider):
    name = "EnvProvider"

    def __init__(self, environ: Mapping[str, str]):
        self.env = environ

    def available(self) -> bool:
        e = self.env
        return bool((e.get("AWS_ACCESS_KEY_ID") or e.get("AWS_ACCESS_KEY")) and (
            e.get("AWS_SECRET_ACCESS_KEY") or e.get("AWS_SECRET_KEY")))

    def fetch(self):
        e = self.env
        akid = e.get("AWS_ACCESS_KEY_ID") or e.get("AWS_ACCESS_KEY") or ""
        secret = e.get("AWS_SECRET_ACCESS_KEY") or e.get("AWS_SECRET_KEY") or ""
        if not akid:
            raise CredentialsError("EnvAccessKeyNotFound: AWS_ACCESS_KEY_ID or AWS_ACCESS_KEY not found in environment")
        if not secret:
            raise CredentialsError("EnvSecretNotFound: AWS_SECRET_ACCESS_KEY or AWS_SECRET_KEY not found in environment")
        return _make(akid, secret, e.get("AWS_SESSION_TOKEN", ""), 0, self.name)


class SharedFileProvider(_Provider):
    name = "SharedCredentialsProvider"

    def __init__(self, environ: Mapping[str, str]):
        self.env = environ
        home = environ.get("HOME") or os.path.expanduser("~")
        self.path = environ.get("AWS_SHARED_CREDENTIALS_FILE") or os.path.join(home, ".aws", "credentials")
        self.profile = environ.get("AWS_PROFILE") or environ.get("AWS_DEFAULT_PROFILE") or "default"

    def _section(self) -> Optional[Mapping[str, str]]:
        if not os.path.exists(self.path):
            return None
        try:
            cp = ini.read(self.path)
        except ini.IniError as e:
            raise CredentialsError(f"SharedCredsLoad: failed to load shared credentials file: {e}")
        if cp is None or not cp.has_section(self.profile):
            return None
        return dict(cp.items(self.profile))

    def available(self) -> bool:
        try:
            sec = self._section()
        except CredentialsError:
            return True  # surface the parse error from fetch()
        return bool(sec and (sec.get("aws_access_key_id") or sec.get("credential_process")))

    def fetch(self):
        sec = self._section()
        if sec is None:
            raise CredentialsError(f"SharedCredsLoad: failed to get profile {self.profile!r} from {self.path}")
        if sec.get("aws_access_key_id"):
            secret = sec.get("aws_secret_access_key", "")
            if not secret:
                raise CredentialsError(
                    f"SharedCredsAccessKey: shared credentials {self.profile} in {self.path} did not contain aws_secret_access_key")
            return _make(sec["aws_access_key_id"], secret, sec.get("aws_session_token", ""), 0, self.name)
        if sec.get("credential_process"):
            return process_credentials(sec["credential_process"])
        raise CredentialsError(f"SharedCredsAccessKey: shared credentials {self.profile} in {self.path} did not contain aws_access_key_id")


def process_credentials(command: str, timeout: float = 60.0):
    """credential_process: runs the command and parses its Version 1 JSON output."""
    try:
        out = subprocess.run(command, shell=True, capture_output=True, timeout=timeout, check=True).stdout
    except (subprocess.SubprocessError, OSError) as e:
        raise CredentialsError(f"ProcessProviderExecutionError: error in credential_process: {e}")
    try:
        j = json.loads(out)
    except ValueError as e:
        raise CredentialsError(f"ProcessProviderParseError: parse failed of process output: {e}")
    if j.get("Version") != 1:
        raise CredentialsError("ProcessProviderVersionError: credential_process output must have Version 1")
    exp = parse_expiration(j["Expiration"]) if j.get("Expiration") else 0
    return _make(j.get("AccessKeyId", ""), j.get("SecretAccessKey", ""), j.get("SessionToken", ""), exp,
                 "ProcessProvider")


# aws-sdk-go v1 endpoints/legacy_regions.go: under the default ("legacy") STS endpoint setting
# these regions resolve STS to the global endpoint sts.amazonaws.com (signed for us-east-1);
# AWS_STS_REGIONAL_ENDPOINTS=regional (or sts_regional_endpoints in the shared config) sends
# them to sts.<region>.<partition suffix> like every other region.
LEGACY_GLOBAL_STS_REGIONS = frozenset({
    "ap-northeast-1", "ap-south-1", "ap-southeast-1", "ap-southeast-2", "ca-central-1", "eu-central-1",
    "eu-north-1", "eu-west-1", "eu-west-2", "eu-west-3", "sa-east-1", "us-east-1", "us-east-2", "us-west-1",
    "us-west-2"})


def session_region(environ: Mapping[str, str], fallback: str = "") -> str:
    """The region ``session.NewSession()`` resolves for its own clients (STS): ``AWS_REGION``;
    with ``AWS_SDK_LOAD_CONFIG`` also ``AWS_DEFAULT_REGION`` and the profile's ``region``.

    The reference applies ``--aws-region`` to the SQS client only (sqs/sqs.go:36), so STS never
    sees it; here it is the fallback when the session has no region (where aws-sdk-go would
    use the global endpoint, which the legacy rule below picks for most regions anyway).
    """
    r = environ.get("AWS_REGION", "")
    if not r and _truthy(environ.get("AWS_SDK_LOAD_CONFIG")):
        r = environ.get("AWS_DEFAULT_REGION", "")
        if not r:
            try:
                prof = environ.get("AWS_PROFILE") or environ.get("AWS_DEFAULT_PROFILE") or "default"
                r = (load_profiles(environ).get(prof) or {}).get("region", "")
            except CredentialsError:
                r = ""
    return r or fallback


def resolve_sts_endpoint(region: str, environ: Mapping[str, str]) -> Tuple[str, str]:
    """(endpoint URL, signing region) for STS as aws-sdk-go v1.35 resolves it."""
    if environ.get("AWS_STS_ENDPOINT"):  # extension: VPC endpoint / test double
        return environ["AWS_STS_ENDPOINT"].rstrip("/"), region or "us-east-1"
    mode = environ.get("AWS_STS_REGIONAL_ENDPOINTS", "").lower()
    if not mode and _truthy(environ.get("AWS_SDK_LOAD_CONFIG")):
        try:
            prof = environ.get("AWS_PROFILE") or environ.get("AWS_DEFAULT_PROFILE") or "default"
            mode = (load_profiles(environ).get(prof) or {}).get("sts_regional_endpoints", "").lower()
        except CredentialsError:
            mode = ""
    if mode and mode not in ("legacy", "regional"):
        # the CLI refuses this at start-up (sqs/session.py), as session.NewSession does
        raise CredentialsError(f"unable to resolve the value of STSRegionalEndpoint for {mode}")
    if not region or (mode != "regional" and region in LEGACY_GLOBAL_STS_REGIONS):
        return "https://sts.amazonaws.com", "us-east-1"
    return f"https://sts.{region}.{native().aws_dns_suffix(region)}", region


class WebIdentityProvider(_Provider):
    """STS AssumeRoleWithWebIdentity (unsigned Query call), the IRSA path on EKS."""

    name = "WebIdentityCredentials"

    def __init__(self, environ: Mapping[str, str], region: str, fetch: Fetch = urllib_fetch, sts_endpoint: str = ""):
        self.token_file = environ.get("AWS_WEB_IDENTITY_TOKEN_FILE", "")
        self.role_arn = environ.get("AWS_ROLE_ARN", "")
        self.session_name = environ.get("AWS_ROLE_SESSION_NAME", "")
        self.region = region
        self.http = fetch
        self.endpoint = sts_endpoint or resolve_sts_endpoint(session_region(environ, region), environ)[0]

    def available(self) -> bool:
        return bool(self.token_file)

    def fetch(self):
        if not self.role_arn:
            raise CredentialsError("WebIdentityErr: role ARN is not set")
        try:
            with open(self.token_file, "r") as f:
                token = f.read().strip()
        except OSError as e:
            raise CredentialsError(f"WebIdentityErr: unable to read file at {self.token_file}: {e}")
        session = self.session_name or f"{int(datetime.now(timezone.utc).timestamp() * 1e9)}"
        form = urllib.parse.urlencode({
            "Action": "AssumeRoleWithWebIdentity",
            "RoleArn": self.role_arn,
            "RoleSessionName": session,
            "Version": "2011-06-15",
            "WebIdentityToken": token,
        }).encode()
        status, body = self.http("POST", self.endpoint + "/", {"Content-Type": "application/x-www-form-urlencoded"},
                                 form, 10.0)
        nat = native()
        text = body.decode(errors="replace")
        if status != 200:
            code = nat.xml_first_text(text, "Code") or f"HTTP {status}"
            msg = nat.xml_first_text(text, "Message") or ""
            raise CredentialsError(f"WebIdentityErr: failed to retrieve credentials: {code}: {msg}")
        akid = nat.xml_first_text(text, "AccessKeyId")
        secret = nat.xml_first_text(text, "SecretAccessKey")
        tok = nat.xml_first_text(text, "SessionToken")
        exp = nat.xml_first_text(text, "Expiration")
        if not akid or not secret:
            raise CredentialsError("WebIdentityErr: STS response carried no credentials")
        return _make(akid, secret, tok or "", parse_expiration(exp) if exp else 0, self.name)


# EKS Pod Identity Agent endpoints (link-local; served by the node's agent).
_POD_IDENTITY_HOSTS = ("169.254.170.23", "fd00:ec2::23")


def _full_uri_error(url: str) -> str:
    """Why ``AWS_CONTAINER_CREDENTIALS_FULL_URI`` may not be used ("" if it may)."""
    import ipaddress

    try:
        u = urllib.parse.urlsplit(url)
        host = u.hostname or ""
    except ValueError as e:
        return f"invalid URL, {e}"
    if not host:
        return "unable to parse host from local HTTP cred provider URL"
    if u.scheme == "https" or host in _POD_IDENTITY_HOSTS:
        return ""
    if host == "localhost":
        return ""
    try:
        if ipaddress.ip_address(host).is_loopback:
            return ""
    except ValueError:
        pass
    return f"invalid endpoint host, {host!r}, only loopback hosts are allowed."


class RemoteProvider(_Provider):
    """ECS container credentials when configured, otherwise EC2 IMDS (v2 with v1 fallback)."""

    def __init__(self, environ: Mapping[str, str], fetch: Fetch = urllib_fetch, imds_endpoint: str = ""):
        self.env = environ
        self.http = fetch
        self.imds = imds_endpoint or environ.get("AWS_EC2_METADATA_SERVICE_ENDPOINT", "") or IMDS_HOST
        self.name = "ECSCredentialsProvider" if self._ecs_url() else "EC2RoleProvider"

    def _ecs_url(self) -> str:
        rel = self.env.get("AWS_CONTAINER_CREDENTIALS_RELATIVE_URI", "")
        if rel:
            return ECS_HOST + rel
        return self.env.get("AWS_CONTAINER_CREDENTIALS_FULL_URI", "")

    def available(self) -> bool:
        return self.env.get("AWS_EC2_METADATA_DISABLED", "").lower() != "true" or bool(self._ecs_url())

    def fetch(self):
        url = self._ecs_url()
        if url:
            if not self.env.get("AWS_CONTAINER_CREDENTIALS_RELATIVE_URI"):
                err = _full_uri_error(url)
                if err:
                    raise CredentialsError(f"CredentialsEndpointError: {err}")
            headers = {}
            token = self.env.get("AWS_CONTAINER_AUTHORIZATION_TOKEN", "")
            token_file = self.env.get("AWS_CONTAINER_AUTHORIZATION_TOKEN_FILE", "")
            if token_file:
                try:
                    with open(token_file) as f:
                        token = f.read().rstrip("\r\n")
                except OSError as e:
                    raise CredentialsError(f"CredentialsEndpointError: failed to read authorization token file: {e}")
            if "\r" in token or "\n" in token:
                raise CredentialsError("CredentialsEndpointError: authorization token contains invalid characters")
            if token:
                headers["Authorization"] = token
            status, body = self.http("GET", url, headers, b"", 5.0)
            if status != 200:
                raise CredentialsError(f"CredentialsEndpointError: failed to load credentials (HTTP {status})")
            return self._parse(body, "CredentialsEndpointError")
        if self.env.get("AWS_EC2_METADATA_DISABLED", "").lower() == "true":
            raise CredentialsError("EC2RoleRequestError: EC2 IMDS access disabled via AWS_EC2_METADATA_DISABLED")
        base = self.imds.rstrip("/")
        headers: Dict[str, str] = {}
        try:
            status, tok = self.http("PUT", base + "/latest/api/token",
                                    {"X-aws-ec2-metadata-token-ttl-seconds": "21600"}, b"", 1.0)
            if status == 200:
                headers["X-aws-ec2-metadata-token"] = tok.decode().strip()
        except OSError:
            pass  # IMDSv1 fallback
        try:
            status, roles = self.http("GET", base + "/latest/meta-data/iam/security-credentials/", headers, b"", 1.0)
        except OSError as e:
            raise CredentialsError(f"NoCredentialProviders: no valid providers in chain ({e})")
        if status != 200 or not roles.strip():
            raise CredentialsError("EC2RoleRequestError: no EC2 instance role found")
        role = roles.decode().splitlines()[0].strip()
        status, body = self.http("GET", base + "/latest/meta-data/iam/security-credentials/" + role, headers, b"", 1.0)
        if status != 200:
            raise CredentialsError(f"EC2RoleRequestError: failed to get {role} EC2 instance role credentials")
        return self._parse(body, "EC2RoleRequestError")

    def _parse(self, body: bytes, err: str):
        """The ECS / IMDS credentials document; anything malformed is a CredentialsError."""
        try:
            j = json.loads(body)
            if j.get("Code", "Success") != "Success":
                raise CredentialsError(f"{err}: {j.get('Code')}: {j.get('Message', '')}")
            return _make(j["AccessKeyId"], j["SecretAccessKey"], j.get("Token", "") or "",
                         parse_expiration(j["Expiration"]) if j.get("Expiration") else 0, self.name)
        except CredentialsError:
            raise
        except (ValueError, KeyError, TypeError, AttributeError) as e:
            raise CredentialsError(f"{err}: malformed credentials response: {e!r}")


def _truthy(v: Optional[str]) -> bool:
    """``AWS_SDK_LOAD_CONFIG``: Go's strconv.ParseBool (aws-sdk-go v1 loadEnvConfig)."""
    from .session import go_parse_bool

    return go_parse_bool(v)


def load_profiles(environ: Mapping[str, str]) -> Dict[str, Dict[str, str]]:
    """Merged shared credentials + (with AWS_SDK_LOAD_CONFIG) shared config profiles.

    Config-file sections are ``[profile name]`` except ``[default]``; credentials-file values
    win, as in aws-sdk-go v1.
    """
    home = environ.get("HOME") or os.path.expanduser("~")
    out: Dict[str, Dict[str, str]] = {}
    if _truthy(environ.get("AWS_SDK_LOAD_CONFIG")):
        cfg_path = environ.get("AWS_CONFIG_FILE") or os.path.join(home, ".aws", "config")
        try:
            cp = ini.read(cfg_path) or ini.IniFile(cfg_path)
        except ini.IniError as e:
            raise CredentialsError(f"SharedConfigLoadError: failed to load config file {cfg_path}: {e}")
        for sec in cp.sections():
            name = sec[len("profile "):].strip() if sec.startswith("profile ") else sec
            out.setdefault(name, {}).update(dict(cp.items(sec)))
    cred_path = environ.get("AWS_SHARED_CREDENTIALS_FILE") or os.path.join(home, ".aws", "credentials")
    try:
        cp = ini.read(cred_path) or ini.IniFile(cred_path)
    except ini.IniError as e:
        raise CredentialsError(f"SharedCredsLoad: failed to load shared credentials file: {e}")
    for sec in cp.sections():
        out.setdefault(sec, {}).update(dict(cp.items(sec)))
    return out


class AssumeRoleProvider(_Provider):
    """``role_arn`` + ``source_profile`` / ``credential_source`` in a shared profile:
    STS ``AssumeRole``, SigV4-signed with the source credentials (aws-sdk-go v1 behaviour)."""

    name = "AssumeRoleProvider"

    def __init__(self, environ: Mapping[str, str], region: str, fetch: Fetch = urllib_fetch, sts_endpoint: str = ""):
        self.env = dict(environ)
        self.profile = environ.get("AWS_PROFILE") or environ.get("AWS_DEFAULT_PROFILE") or "default"
        self.region = region
        self.http = fetch
        self.sts_endpoint = sts_endpoint

    def _section(self) -> Optional[Dict[str, str]]:
        try:
            return load_profiles(self.env).get(self.profile)
        except CredentialsError:
            return None

    def available(self) -> bool:
        sec = self._section()
        return bool(sec and sec.get("role_arn") and not sec.get("aws_access_key_id"))

    def _source(self, sec: Dict[str, str]):
        if sec.get("source_profile"):
            src_env = dict(self.env)
            src_env["AWS_PROFILE"] = sec["source_profile"]
            profiles = load_profiles(self.env)
            src = profiles.get(sec["source_profile"])
            if src is None:
                raise CredentialsError(f"SharedConfigAssumeRoleError: source profile {sec['source_profile']} not found")
            if src.get("role_arn") and not src.get("aws_access_key_id"):
                if sec["source_profile"] == self.profile:
                    raise CredentialsError("SharedConfigAssumeRoleError: source_profile refers to itself")
                return AssumeRoleProvider(src_env, self.region, self.http, self.sts_endpoint).fetch()  # role chaining
            if src.get("aws_access_key_id"):
                return _make(src["aws_access_key_id"], src.get("aws_secret_access_key", ""), src.get("aws_session_token", ""),
                             0, "SharedCredentialsProvider")
            if src.get("credential_process"):
                return process_credentials(src["credential_process"])
            raise CredentialsError(f"SharedConfigAssumeRoleError: source profile {sec['source_profile']} has no credentials")
        cs = sec.get("credential_source", "")
        if cs == "Environment":
            return EnvProvider(self.env).fetch()
        if cs in ("Ec2InstanceMetadata", "EcsContainer"):
            return RemoteProvider(self.env, self.http).fetch()
        raise CredentialsError("SharedConfigAssumeRoleError: role_arn needs source_profile or credential_source")

    def fetch(self):
        nat = native()
        sec = self._section() or {}
        src = self._source(sec)
        if self.sts_endpoint:
            endpoint, region = self.sts_endpoint, self.region or "us-east-1"
        else:
            endpoint, region = resolve_sts_endpoint(session_region(self.env, self.region), self.env)
        params = {"Action": "AssumeRole", "RoleArn": sec["role_arn"], "Version": "2011-06-15",
                  "RoleSessionName": sec.get("role_session_name") or f"{int(datetime.now(timezone.utc).timestamp() * 1e9)}"}
        if sec.get("external_id"):
            params["ExternalId"] = sec["external_id"]
        if sec.get("duration_seconds"):
            params["DurationSeconds"] = sec["duration_seconds"]
        body = "&".join(f"{nat.aws_uri_encode(k, False)}={nat.aws_uri_encode(v, False)}" for k, v in sorted(params.items()))
        host = urllib.parse.urlsplit(endpoint).netloc
        headers = [("Host", host), ("Content-Type", "application/x-www-form-urlencoded; charset=utf-8")]
        signer = nat.SigV4Signer(region, "sts")
        signed, _ = signer.sign(src, int(datetime.now(timezone.utc).timestamp() * 1e9), "POST", "/", "", headers, body.encode())
        status, resp = self.http("POST", endpoint + "/", {k: v for k, v in signed if k != "Host"}, body.encode(), 10.0)
        text = resp.decode(errors="replace")
        if status != 200:
            code = nat.xml_first_text(text, "Code") or f"HTTP {status}"
            raise CredentialsError(f"AssumeRoleError: {code}: {nat.xml_first_text(text, 'Message') or ''}")
        akid, secret = nat.xml_first_text(text, "AccessKeyId"), nat.xml_first_text(text, "SecretAccessKey")
        if not akid or not secret:
            raise CredentialsError("AssumeRoleError: STS response carried no credentials")
        exp = nat.xml_first_text(text, "Expiration")
        return _make(akid, secret, nat.xml_first_text(text, "SessionToken") or "", parse_expiration(exp) if exp else 0,
                     self.name)


def default_chain(environ: Optional[Mapping[str, str]] = None, region: str = "", fetch: Fetch = urllib_fetch) -> List[_Provider]:
    env = dict(os.environ if environ is None else environ)
    return [EnvProvider(env), WebIdentityProvider(env, region, fetch), AssumeRoleProvider(env, region, fetch),
            SharedFileProvider(env), RemoteProvider(env, fetch)]


def make_chain_provider(providers: Optional[List[_Provider]] = None, environ: Optional[Mapping[str, str]] = None,
                        region: str = "", fetch: Fetch = urllib_fetch):
    """A native ``CredentialsProvider`` backed by the chain (first available provider wins)."""
    nat = native()
    chain = providers if providers is not None else default_chain(environ, region, fetch)

    class ChainProvider(nat.CredentialsProvider):
        def __init__(self) -> None:
            super().__init__()
            self.providers = chain
            self.lock = threading.Lock()
            self.last_provider = ""

        def retrieve(self):
            with self.lock:
                errors = []
                for p in self.providers:
                    if hasattr(p, "available") and not p.available():
                        continue
                    try:
                        c = p.fetch()
                    except CredentialsError as e:
                        errors.append(str(e))
                        # env/web-identity/shared are authoritative once configured (SDK behaviour)
                        if not isinstance(p, RemoteProvider):
                            raise
                        continue
                    self.last_provider = p.name
                    return c
                raise CredentialsError(
                    "NoCredentialProviders: no valid providers in chain. Deprecated.\n\tFor verbose messaging see "
                    "aws.Config.CredentialsChainVerboseErrors" + (f" ({'; '.join(errors)})" if errors else ""))

    return ChainProvider()


def static_provider(akid: str, secret: str, token: str = ""):
    nat = native()
    return nat.StaticCredentialsProvider(nat.Credentials(akid, secret, token, 0, "StaticProvider"))

"""AWS credential chain (aws-sdk-go v1 session defaults the reference relies on, sqs/sqs.go:36)."""
import json

import pytest

from kube_sqs_autoscaler_amd.sqs import credentials as cr


def chain(env, fetch=None, region="us-east-1"):
    return cr.make_chain_provider(environ=env, region=region, fetch=fetch or (lambda *a: (404, b"")))


def test_env_credentials(nat):
    c = chain({"AWS_ACCESS_KEY_ID": "AK", "AWS_SECRET_ACCESS_KEY": "SK", "AWS_SESSION_TOKEN": "T"}).retrieve()
    assert (c.access_key_id, c.secret_access_key, c.session_token, c.provider_name) == ("AK", "SK", "T", "EnvProvider")
    c = chain({"AWS_ACCESS_KEY": "AK2", "AWS_SECRET_KEY": "SK2"}).retrieve()
    assert c.access_key_id == "AK2"


def test_shared_file_profiles(tmp_path, nat):
    f = tmp_path / "credentials"
    f.write_text("[default]\naws_access_key_id = D\naws_secret_access_key = DS\n\n[prod]\naws_access_key_id=P\naws_secret_access_key=PS\naws_session_token=PT\n")
    env = {"AWS_SHARED_CREDENTIALS_FILE": str(f)}
    assert chain(env).retrieve().access_key_id == "D"
    c = chain({**env, "AWS_PROFILE": "prod"}).retrieve()
    assert (c.access_key_id, c.session_token, c.provider_name) == ("P", "PT", "SharedCredentialsProvider")
    with pytest.raises(Exception, match="aws_secret_access_key"):
        f.write_text("[default]\naws_access_key_id = D\n")
        chain(env).retrieve()


def test_env_beats_shared_file(tmp_path, nat):
    f = tmp_path / "credentials"
    f.write_text("[default]\naws_access_key_id = D\naws_secret_access_key = DS\n")
    env = {"AWS_SHARED_CREDENTIALS_FILE": str(f), "AWS_ACCESS_KEY_ID": "E", "AWS_SECRET_ACCESS_KEY": "ES"}
    assert chain(env).retrieve().access_key_id == "E"


def test_credential_process(tmp_path, nat):
    out = {"Version": 1, "AccessKeyId": "CP", "SecretAccessKey": "CPS", "SessionToken": "CPT",
           "Expiration": "2030-01-01T00:00:00Z"}
    script = tmp_path / "proc.sh"
    script.write_text("#!/bin/sh\necho '" + json.dumps(out) + "'\n")
    script.chmod(0o755)
    f = tmp_path / "credentials"
    f.write_text(f"[default]\ncredential_process = {script}\n")
    c = chain({"AWS_SHARED_CREDENTIALS_FILE": str(f)}).retrieve()
    assert c.access_key_id == "CP" and c.expires_unix_ns == cr.parse_expiration("2030-01-01T00:00:00Z")


def test_web_identity(tmp_path, nat):
    tok = tmp_path / "token"
    tok.write_text("jwt-token\n")
    seen = {}

    def fetch(method, url, headers, body, timeout):
        seen.update(method=method, url=url, body=body.decode())
        return 200, (b"<AssumeRoleWithWebIdentityResponse><AssumeRoleWithWebIdentityResult><Credentials>"
                     b"<AccessKeyId>ASIAWEB</AccessKeyId><SecretAccessKey>WS</SecretAccessKey>"
                     b"<SessionToken>WT</SessionToken><Expiration>2031-02-03T04:05:06Z</Expiration>"
                     b"</Credentials></AssumeRoleWithWebIdentityResult></AssumeRoleWithWebIdentityResponse>")

    env = {"AWS_WEB_IDENTITY_TOKEN_FILE": str(tok), "AWS_ROLE_ARN": "arn:aws:iam::1:role/r", "AWS_ROLE_SESSION_NAME": "s"}
    c = chain(env, fetch, region="us-west-2").retrieve()
    assert (c.access_key_id, c.secret_access_key, c.session_token) == ("ASIAWEB", "WS", "WT")
    # us-west-2 is a legacy-global STS region in aws-sdk-go v1: the default resolves to sts.amazonaws.com
    assert seen["url"] == "https://sts.amazonaws.com/" and "Action=AssumeRoleWithWebIdentity" in seen["body"]
    assert "WebIdentityToken=jwt-token" in seen["body"] and "RoleArn=arn%3Aaws%3Aiam%3A%3A1%3Arole%2Fr" in seen["body"]


def test_web_identity_error(tmp_path, nat):
    tok = tmp_path / "token"
    tok.write_text("t")
    fetch = lambda *a: (403, b"<ErrorResponse><Error><Code>AccessDenied</Code><Message>nope</Message></Error></ErrorResponse>")
    with pytest.raises(Exception, match="AccessDenied: nope"):
        chain({"AWS_WEB_IDENTITY_TOKEN_FILE": str(tok), "AWS_ROLE_ARN": "a"}, fetch).retrieve()


def test_ecs_container_credentials(nat):
    def fetch(method, url, headers, body, timeout):
        assert url == "http://169.254.170.2/v2/credentials/abc" and headers.get("Authorization") == "Bearer x"
        return 200, json.dumps({"AccessKeyId": "ECS", "SecretAccessKey": "S", "Token": "T", "Expiration": "2030-01-01T00:00:00Z"}).encode()

    c = chain({"AWS_CONTAINER_CREDENTIALS_RELATIVE_URI": "/v2/credentials/abc", "AWS_CONTAINER_AUTHORIZATION_TOKEN": "Bearer x"}, fetch).retrieve()
    assert c.access_key_id == "ECS" and c.provider_name == "ECSCredentialsProvider"


def test_imds_v2(nat):
    calls = []

    def fetch(method, url, headers, body, timeout):
        calls.append((method, url, dict(headers)))
        if url.endswith("/latest/api/token"):
            return 200, b"imds-token"
        if url.endswith("/security-credentials/"):
            assert headers["X-aws-ec2-metadata-token"] == "imds-token"
            return 200, b"node-role\n"
        if url.endswith("/security-credentials/node-role"):
            return 200, json.dumps({"Code": "Success", "AccessKeyId": "EC2", "SecretAccessKey": "S", "Token": "T",
                                    "Expiration": "2030-01-01T00:00:00Z"}).encode()
        return 404, b""

    c = chain({}, fetch).retrieve()
    assert c.access_key_id == "EC2" and c.provider_name == "EC2RoleProvider"
    assert calls[0][0] == "PUT" and calls[0][2]["X-aws-ec2-metadata-token-ttl-seconds"] == "21600"


def test_no_credentials(nat):
    with pytest.raises(Exception, match="NoCredentialProviders"):
        chain({"AWS_EC2_METADATA_DISABLED": "true"}).retrieve()


def test_parse_expiration():
    assert cr.parse_expiration("1970-01-01T00:00:01Z") == 10**9
    assert cr.parse_expiration("1970-01-01T01:00:00+01:00") == 0
    assert cr.parse_expiration("1970-01-01T00:00:00.5Z") == 5 * 10**8


def test_chain_feeds_native_signer_lazily_and_caches(nat):
    """The native client asks the Python chain only when its cache is cold."""
    calls = []

    class P(cr._Provider):
        name = "counting"

        def available(self):
            return True

        def fetch(self):
            calls.append(1)
            return nat.Credentials("AKIDTEST", "secret/KEY", "", 0, "counting")

    s = nat.FakeSqsServer()
    s.require_signature("AKIDTEST", "secret/KEY", "eu-west-1")
    s.start()
    try:
        from kube_sqs_autoscaler_amd.autoscaler import new_sqs_api

        api = new_sqs_api("eu-west-1", nat.RealClock(), endpoint=s.url, credentials=cr.make_chain_provider([P()]))
        assert calls == []  # lazy, like session.NewSession
        url = s.url + "/1/q"
        s.set_attributes(url, {"A": "1"})
        c = nat.SqsClient(api, url, ["A"])
        assert c.num_messages() == 1 and c.num_messages() == 1
        assert len(calls) == 1 and s.signature_failures() == 0
    finally:
        s.stop()


def test_assume_role_from_shared_config(tmp_path, nat):
    (tmp_path / "credentials").write_text("[base]\naws_access_key_id = AKIDBASE\naws_secret_access_key = basesecret\n")
    (tmp_path / "config").write_text("[profile deploy]\nrole_arn = arn:aws:iam::123:role/ksa\nsource_profile = base\n"
                                     "external_id = ext-1\nrole_session_name = ksa-session\n")
    seen = {}

    def fetch(method, url, headers, body, timeout):
        seen.update(url=url, headers=headers, body=body.decode())
        return 200, (b"<AssumeRoleResponse><AssumeRoleResult><Credentials><AccessKeyId>ASIAROLE</AccessKeyId>"
                     b"<SecretAccessKey>RS</SecretAccessKey><SessionToken>RT</SessionToken>"
                     b"<Expiration>2031-01-01T00:00:00Z</Expiration></Credentials></AssumeRoleResult></AssumeRoleResponse>")

    env = {"AWS_SHARED_CREDENTIALS_FILE": str(tmp_path / "credentials"), "AWS_CONFIG_FILE": str(tmp_path / "config"),
           "AWS_SDK_LOAD_CONFIG": "1", "AWS_PROFILE": "deploy"}
    c = chain(env, fetch, region="eu-west-1").retrieve()
    assert (c.access_key_id, c.session_token, c.provider_name) == ("ASIAROLE", "RT", "AssumeRoleProvider")
    assert seen["url"] == "https://sts.amazonaws.com/"  # legacy-global region, default setting
    assert "Action=AssumeRole" in seen["body"] and "ExternalId=ext-1" in seen["body"] and "RoleSessionName=ksa-session" in seen["body"]
    auth = seen["headers"]["Authorization"]
    assert auth.startswith("AWS4-HMAC-SHA256 Credential=AKIDBASE/") and "/us-east-1/sts/aws4_request" in auth
    seen.clear()
    chain({**env, "AWS_STS_REGIONAL_ENDPOINTS": "regional"}, fetch, region="eu-west-1").retrieve()
    assert seen["url"] == "https://sts.eu-west-1.amazonaws.com/"
    assert "/eu-west-1/sts/aws4_request" in seen["headers"]["Authorization"]


def test_assume_role_needs_sdk_load_config(tmp_path, nat):
    (tmp_path / "config").write_text("[profile deploy]\nrole_arn = arn:aws:iam::123:role/ksa\nsource_profile = base\n")
    env = {"AWS_CONFIG_FILE": str(tmp_path / "config"), "AWS_PROFILE": "deploy", "AWS_EC2_METADATA_DISABLED": "true",
           "AWS_SHARED_CREDENTIALS_FILE": str(tmp_path / "none")}
    with pytest.raises(Exception, match="NoCredentialProviders"):
        chain(env).retrieve()  # aws-sdk-go v1 ignores ~/.aws/config without AWS_SDK_LOAD_CONFIG


def test_assume_role_error(tmp_path, nat):
    (tmp_path / "credentials").write_text("[base]\naws_access_key_id = A\naws_secret_access_key = S\n"
                                          "[deploy]\nrole_arn = arn:aws:iam::1:role/r\nsource_profile = base\n")
    fetch = lambda *a: (403, b"<ErrorResponse><Error><Code>AccessDenied</Code><Message>not allowed</Message></Error></ErrorResponse>")
    env = {"AWS_SHARED_CREDENTIALS_FILE": str(tmp_path / "credentials"), "AWS_PROFILE": "deploy"}
    with pytest.raises(Exception, match="AccessDenied: not allowed"):
        chain(env, fetch).retrieve()


@pytest.mark.parametrize("env,flag,want", [
    ({}, "us-west-2", ("https://sts.amazonaws.com", "us-east-1")),           # legacy-global region
    ({}, "ap-east-1", ("https://sts.ap-east-1.amazonaws.com", "ap-east-1")),  # not in the legacy list
    ({}, "", ("https://sts.amazonaws.com", "us-east-1")),                     # no region: global
    ({"AWS_STS_REGIONAL_ENDPOINTS": "regional"}, "us-west-2", ("https://sts.us-west-2.amazonaws.com", "us-west-2")),
    ({"AWS_REGION": "eu-central-1", "AWS_STS_REGIONAL_ENDPOINTS": "regional"}, "us-west-2",
     ("https://sts.eu-central-1.amazonaws.com", "eu-central-1")),           # the session region wins over the flag
    ({"AWS_DEFAULT_REGION": "ap-east-1"}, "", ("https://sts.amazonaws.com", "us-east-1")),  # only with LOAD_CONFIG
    ({"AWS_DEFAULT_REGION": "ap-east-1", "AWS_SDK_LOAD_CONFIG": "1"}, "", ("https://sts.ap-east-1.amazonaws.com", "ap-east-1")),
    ({}, "cn-north-1", ("https://sts.cn-north-1.amazonaws.com.cn", "cn-north-1")),
    ({}, "us-gov-west-1", ("https://sts.us-gov-west-1.amazonaws.com", "us-gov-west-1")),
    ({"AWS_STS_ENDPOINT": "https://vpce-1.sts.example/"}, "eu-west-1", ("https://vpce-1.sts.example", "eu-west-1")),
])
def test_sts_endpoint_resolution(nat, env, flag, want):
    """aws-sdk-go v1.35 STS endpoint rules (endpoints/legacy_regions.go, AWS_STS_REGIONAL_ENDPOINTS)."""
    assert cr.resolve_sts_endpoint(cr.session_region(env, flag), env) == want


def test_sts_regional_endpoints_from_shared_config(tmp_path, nat):
    (tmp_path / "config").write_text("[default]\nsts_regional_endpoints = regional\nregion = eu-west-2\n")
    env = {"AWS_CONFIG_FILE": str(tmp_path / "config"), "AWS_SHARED_CREDENTIALS_FILE": str(tmp_path / "none"),
           "AWS_SDK_LOAD_CONFIG": "true"}
    assert cr.resolve_sts_endpoint(cr.session_region(env, "us-east-1"), env) == ("https://sts.eu-west-2.amazonaws.com", "eu-west-2")


@pytest.mark.parametrize("body", [b"not json", b"[]", b'{"AccessKeyId": "A"}', b'{"Code": "Failure", "Message": "no role"}'])
def test_malformed_remote_credentials_are_credential_errors(nat, body):
    """A broken ECS / IMDS credentials document surfaces as a CredentialsError (logged per poll),
    never as a stray exception from the provider chain."""
    def fetch(method, url, headers, b, timeout):
        return 200, body

    p = cr.RemoteProvider({"AWS_CONTAINER_CREDENTIALS_FULL_URI": "http://169.254.170.2/creds"}, fetch)
    with pytest.raises(cr.CredentialsError):
        p.fetch()


@pytest.mark.parametrize("url,ok", [
    ("http://127.0.0.1:51679/creds", True), ("http://localhost/creds", True), ("http://[::1]/creds", True),
    ("http://169.254.170.23/v1/credentials", True), ("http://[fd00:ec2::23]/v1/credentials", True),
    ("https://creds.example.com/role", True), ("http://10.0.0.8/creds", False), ("http://169.254.170.2/creds", False),
])
def test_full_uri_host_rules(nat, url, ok):
    """A plain-http FULL_URI must be loopback (or the EKS Pod Identity Agent); anything else is
    refused before a request is sent."""
    sent = []

    def fetch(method, u, headers, body, timeout):
        sent.append(u)
        return 200, json.dumps({"AccessKeyId": "F", "SecretAccessKey": "S", "Token": "T",
                                "Expiration": "2030-01-01T00:00:00Z"}).encode()

    p = cr.RemoteProvider({"AWS_CONTAINER_CREDENTIALS_FULL_URI": url}, fetch)
    if ok:
        assert p.fetch().access_key_id == "F" and sent == [url]
    else:
        with pytest.raises(cr.CredentialsError, match="only loopback hosts are allowed"):
            p.fetch()
        assert sent == []


def test_eks_pod_identity_token_file_is_reread(nat, tmp_path):
    """EKS Pod Identity: the agent's token is read from AWS_CONTAINER_AUTHORIZATION_TOKEN_FILE on
    every fetch (it rotates) and wins over AWS_CONTAINER_AUTHORIZATION_TOKEN."""
    tok = tmp_path / "eks-pod-identity-token"
    tok.write_text("token-1")
    seen = []

    def fetch(method, url, headers, body, timeout):
        seen.append(headers.get("Authorization"))
        return 200, json.dumps({"AccessKeyId": "POD", "SecretAccessKey": "S", "Token": "T",
                                "Expiration": "2030-01-01T00:00:00Z"}).encode()

    env = {"AWS_CONTAINER_CREDENTIALS_FULL_URI": "http://169.254.170.23/v1/credentials",
           "AWS_CONTAINER_AUTHORIZATION_TOKEN_FILE": str(tok), "AWS_CONTAINER_AUTHORIZATION_TOKEN": "inline"}
    c = chain(env, fetch).retrieve()
    assert c.access_key_id == "POD" and c.provider_name == "ECSCredentialsProvider"
    tok.write_text("token-2\n")
    cr.RemoteProvider(env, fetch).fetch()
    assert seen == ["token-1", "token-2"]
    tok.unlink()
    with pytest.raises(cr.CredentialsError, match="token file"):
        cr.RemoteProvider(env, fetch).fetch()

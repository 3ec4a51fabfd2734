"""Queue-depth source: /root/reference/sqs/sqs_test.go + attribute-summing edge cases (sqs.go:45-67)."""
import pytest

DEFAULT = ["ApproximateNumberOfMessages", "ApproximateNumberOfMessagesDelayed", "ApproximateNumberOfMessagesNotVisible"]


def mock_sqs_client(nat, attrs=None):
    """NewMockSqsClient (sqs_test.go:43-59): starts at 10/10/10."""
    api = nat.MockSqsApi(attrs or {n: "10" for n in DEFAULT})
    return nat.SqsClient(api, "example.com", list(DEFAULT)), api


def test_new_sqs_client(nat):  # sqs_test.go:11-17
    from kube_sqs_autoscaler_amd.autoscaler import new_sqs_api, new_sqs_client
    from kube_sqs_autoscaler_amd.config import TargetConfig
    from kube_sqs_autoscaler_amd.sqs.credentials import static_provider

    api = new_sqs_api("us-east-1", nat.RealClock(), credentials=static_provider("a", "b"))
    c = new_sqs_client(TargetConfig(queue_url="example.com", attribute_names=list(DEFAULT)), api)
    assert c.queue_url == "example.com" and c.attribute_names == DEFAULT
    assert api.endpoint() == "https://sqs.us-east-1.amazonaws.com"


def test_num_messages(nat):  # sqs_test.go:19-25
    c, _ = mock_sqs_client(nat)
    assert c.num_messages() == 30


def test_default_attribute_names(nat):  # sqs.go:26-33
    assert nat.default_attribute_names() == DEFAULT


def test_only_requested_attributes_are_summed(nat):
    api = nat.MockSqsApi({"ApproximateNumberOfMessages": "7", "ApproximateNumberOfMessagesDelayed": "1000",
                          "ApproximateNumberOfMessagesNotVisible": "5"})
    c = nat.SqsClient(api, "q", ["ApproximateNumberOfMessages", "ApproximateNumberOfMessagesNotVisible"])
    assert c.num_messages() == 12


@pytest.mark.parametrize("value,expect", [("+5", 5), ("-3", -3), ("007", 7), ("9223372036854775807", 2**63 - 1)])
def test_atoi_forms(nat, value, expect):
    c, _ = mock_sqs_client(nat, {"A": value})
    c = nat.SqsClient(nat.MockSqsApi({"A": value}), "q", ["A"])
    assert c.num_messages() == expect


def test_sum_wraps_like_go_int(nat):
    big = str(2**63 - 1)
    c = nat.SqsClient(nat.MockSqsApi({"A": big, "B": "1"}), "q", ["A", "B"])
    assert c.num_messages() == -(2**63)


@pytest.mark.parametrize("value,msg", [
    ("abc", "Failed to get 'A' number of messages in queue: strconv.Atoi: parsing \"abc\": invalid syntax"),
    ("", "Failed to get 'A' number of messages in queue: strconv.Atoi: parsing \"\": invalid syntax"),
    ("1_000", "Failed to get 'A' number of messages in queue: strconv.Atoi: parsing \"1_000\": invalid syntax"),
    ("99999999999999999999", "Failed to get 'A' number of messages in queue: strconv.Atoi: parsing \"99999999999999999999\": value out of range"),
])
def test_non_integer_attribute_errors(nat, value, msg):
    c = nat.SqsClient(nat.MockSqsApi({"A": value}), "q", ["A"])
    with pytest.raises(nat.NativeError) as e:
        c.num_messages()
    assert str(e.value) == msg


def test_missing_attribute_is_an_error_not_a_panic(nat):
    # the reference dereferences a nil *string here (sqs.go:58) and crash-loops; documented deviation
    c = nat.SqsClient(nat.MockSqsApi({"A": "1"}), "q", ["A", ""])
    with pytest.raises(nat.NativeError, match="Failed to get '' number of messages in queue"):
        c.num_messages()


def test_api_error_is_wrapped(nat):
    c, api = mock_sqs_client(nat)
    api.fail_next(1, "RequestError: send request failed")
    with pytest.raises(nat.NativeError, match="^Failed to get messages in SQS: RequestError: send request failed$"):
        c.num_messages()
    assert c.num_messages() == 30


def test_python_sqs_api_plugs_into_native_client(nat):
    class Api(nat.SqsApi):
        def get_queue_attributes(self, url, names):
            assert url == "q" and names == ["A", "B"]
            return {"A": "2", "B": "3"}

    assert nat.SqsClient(Api(), "q", ["A", "B"]).num_messages() == 5


@pytest.mark.parametrize("region,endpoint,signing", [
    ("us-east-1", "https://sqs.us-east-1.amazonaws.com", "us-east-1"),
    ("us-gov-west-1", "https://sqs.us-gov-west-1.amazonaws.com", "us-gov-west-1"),
    ("cn-northwest-1", "https://sqs.cn-northwest-1.amazonaws.com.cn", "cn-northwest-1"),
    ("us-iso-east-1", "https://sqs.us-iso-east-1.c2s.ic.gov", "us-iso-east-1"),
    ("us-isob-east-1", "https://sqs.us-isob-east-1.sc2s.sgov.gov", "us-isob-east-1"),
    ("fips-us-west-2", "https://sqs-fips.us-west-2.amazonaws.com", "us-west-2"),
    ("", "", ""),
])
def test_endpoint_partitions(nat, region, endpoint, signing):
    """aws-sdk-go v1 endpoint resolution for "sqs" (partition by region pattern; fips-<region>
    pseudo-regions sign for <region>)."""
    assert nat.HttpSqsApi.endpoint_for_region(region) == endpoint
    assert nat.HttpSqsApi.signing_region(region) == signing


def test_fips_region_signs_for_base_region(nat):
    from kube_sqs_autoscaler_amd.autoscaler import new_sqs_api
    from kube_sqs_autoscaler_amd.sqs.credentials import static_provider

    s = nat.FakeSqsServer()
    s.require_signature("AKID", "SECRET", "us-east-1")
    s.start()
    try:
        api = new_sqs_api("fips-us-east-1", nat.RealClock(), endpoint=s.url, credentials=static_provider("AKID", "SECRET"))
        url = s.url + "/1/q"
        s.set_attributes(url, {n: "1" for n in DEFAULT})
        assert nat.SqsClient(api, url, list(DEFAULT)).num_messages() == 3
        assert s.signature_failures() == 0
    finally:
        s.stop()

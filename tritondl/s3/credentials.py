"""Credential providers — reference ``EnvGeneric``
(``internal/uploader/minio_credential_provider.go:16-43``, component C9a)
chained with minio-go's ``EnvAWS`` and ``EnvMinio`` exactly as
``uploader.go:45-49`` does.

Chain semantics (minio-go ``Chain.Retrieve``): providers are tried in
order, a provider yielding neither an access key nor a secret is skipped,
and if every provider is empty the request is anonymous.
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Mapping, Sequence

SIGNATURE_V4 = "v4"
SIGNATURE_ANONYMOUS = "anonymous"


@dataclass
class Value:
    access_key_id: str = ""
    secret_access_key: str = ""
    session_token: str = ""
    signer_type: str = SIGNATURE_ANONYMOUS

    @property
    def anonymous(self) -> bool:
        return self.signer_type == SIGNATURE_ANONYMOUS


class Provider:
    def retrieve(self) -> Value:  # pragma: no cover - interface
        raise NotImplementedError

    def is_expired(self) -> bool:
        return False


class EnvGeneric(Provider):
    """``S3_ACCESS_KEY`` / ``S3_SECRET_KEY``; SigV4 only if BOTH are set,
    otherwise anonymous.  Never errors; expired until first retrieve."""

    def __init__(self, env: Mapping[str, str] | None = None) -> None:
        self.env = env
        self.retrieved = False

    def retrieve(self) -> Value:
        env = os.environ if self.env is None else self.env
        self.retrieved = False
        ak, sk = env.get("S3_ACCESS_KEY", ""), env.get("S3_SECRET_KEY", "")
        st = SIGNATURE_V4 if ak and sk else SIGNATURE_ANONYMOUS
        self.retrieved = True
        return Value(ak, sk, "", st)

    def is_expired(self) -> bool:
        return not self.retrieved


class EnvAWS(Provider):
    def __init__(self, env: Mapping[str, str] | None = None) -> None:
        self.env = env

    def retrieve(self) -> Value:
        env = os.environ if self.env is None else self.env
        ak = env.get("AWS_ACCESS_KEY_ID", "") or env.get("AWS_ACCESS_KEY", "")
        sk = env.get("AWS_SECRET_ACCESS_KEY", "") or env.get("AWS_SECRET_KEY", "")
        st = SIGNATURE_V4 if ak and sk else SIGNATURE_ANONYMOUS
        return Value(ak, sk, env.get("AWS_SESSION_TOKEN", ""), st)


class EnvMinio(Provider):
    def __init__(self, env: Mapping[str, str] | None = None) -> None:
        self.env = env

    def retrieve(self) -> Value:
        env = os.environ if self.env is None else self.env
        ak, sk = env.get("MINIO_ACCESS_KEY", ""), env.get("MINIO_SECRET_KEY", "")
        st = SIGNATURE_V4 if ak and sk else SIGNATURE_ANONYMOUS
        return Value(ak, sk, "", st)


class Static(Provider):
    def __init__(self, access_key: str, secret_key: str, session_token: str = "") -> None:
        self.v = Value(access_key, secret_key, session_token,
                       SIGNATURE_V4 if access_key and secret_key else SIGNATURE_ANONYMOUS)

    def retrieve(self) -> Value:
        return self.v


class Chain(Provider):
    def __init__(self, providers: Sequence[Provider]) -> None:
        self.providers = list(providers)
        self._cur: Provider | None = None

    def retrieve(self) -> Value:
        for p in self.providers:
            v = p.retrieve()
            if not v.access_key_id and not v.secret_access_key:
                continue
            self._cur = p
            return v
        self._cur = None
        return Value()

    def is_expired(self) -> bool:
        return self._cur is None or self._cur.is_expired()


def default_chain(env: Mapping[str, str] | None = None) -> Chain:
    """``credentials.NewChainCredentials([EnvGeneric, EnvAWS, EnvMinio])``."""
    return Chain([EnvGeneric(env), EnvAWS(env), EnvMinio(env)])

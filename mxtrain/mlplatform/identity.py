"""Identity and certificates for the node's web services (replaces Dex + oauth2-proxy
(C40), the Istio ingress auth (C39) and cert-manager (C38); reference:
charts/ml-platform/kubeflow-{dex,oauth2-proxy,istio,cert-manager}).

* Static-password identity provider (Dex ``staticPasswords``): users in
  ``$MXTRAIN_HOME/identity/users.yaml`` (email, PBKDF2-SHA256 hash, groups); an OIDC-shaped
  password-grant token endpoint issuing HS256 JWTs (``iss``/``sub``/``email``/``groups``/
  ``iat``/``exp``) signed with a node-local key (0600), discovery document, userinfo.
* oauth2-proxy role: ``verify_token`` checks signature, issuer and expiry; the dashboard
  accepts ``Authorization: Bearer <jwt>`` or the ``mxtrain_session`` cookie and acts as
  that user (profile roles, mlplatform/profiles.py ``can``).
* cert-manager role: ``issue_cert`` keeps a node CA and issues / renews server
  certificates (openssl CLI) with DNS / IP SANs; renewal when < ``renew_days`` remain.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import os
import secrets
import subprocess
import time
from typing import Dict, List, Optional

import yaml

ISSUER = "mxtrain-dex"


def _home() -> str:
    from ..runtime.storage import mxtrain_home
    return os.path.join(mxtrain_home(), "identity")


def _b64(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def _unb64(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


# ------------------------------------------------------------------------------- users
def hash_password(password: str, salt: Optional[bytes] = None, rounds: int = 200_000) -> str:
    salt = salt or secrets.token_bytes(16)
    dk = hashlib.pbkdf2_hmac("sha256", password.encode(), salt, rounds)
    return f"pbkdf2-sha256${rounds}${_b64(salt)}${_b64(dk)}"


def check_password(password: str, stored: str) -> bool:
    try:
        kind, rounds, salt, dk = stored.split("$")
    except ValueError:
        return False
    if kind != "pbkdf2-sha256":
        return False
    got = hashlib.pbkdf2_hmac("sha256", password.encode(), _unb64(salt), int(rounds))
    return hmac.compare_digest(got, _unb64(dk))


def _users_path() -> str:
    return os.path.join(_home(), "users.yaml")


def load_users() -> Dict[str, dict]:
    p = _users_path()
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        doc = yaml.safe_load(f) or {}
    return {u["email"]: u for u in doc.get("staticPasswords") or []}


def add_user(email: str, password: str, groups: Optional[List[str]] = None) -> dict:
    users = load_users()
    users[email] = {"email": email, "hash": hash_password(password), "username": email.split("@")[0],
                    "groups": list(groups or [])}
    os.makedirs(_home(), exist_ok=True)
    fd = os.open(_users_path(), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    with os.fdopen(fd, "w") as f:
        yaml.safe_dump({"staticPasswords": list(users.values())}, f)
    return {"email": email, "groups": users[email]["groups"]}


# ------------------------------------------------------------------------------- tokens
def _signing_key() -> bytes:
    p = os.path.join(_home(), "signing.key")
    if not os.path.exists(p):
        os.makedirs(_home(), exist_ok=True)
        fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
        with os.fdopen(fd, "wb") as f:
            f.write(secrets.token_bytes(32))
    with open(p, "rb") as f:
        return f.read()


def issue_token(email: str, ttl: int = 3600, groups: Optional[List[str]] = None) -> str:
    now = int(time.time())
    head = _b64(json.dumps({"alg": "HS256", "typ": "JWT"}, separators=(",", ":")).encode())
    body = _b64(json.dumps({"iss": ISSUER, "sub": email, "email": email, "groups": list(groups or []),
                            "iat": now, "exp": now + int(ttl)}, separators=(",", ":")).encode())
    sig = hmac.new(_signing_key(), f"{head}.{body}".encode(), hashlib.sha256).digest()
    return f"{head}.{body}.{_b64(sig)}"


def verify_token(token: str) -> dict:
    """Claims of a valid token; PermissionError otherwise (bad shape / signature / issuer /
    algorithm, expired)."""
    try:
        head, body, sig = token.split(".")
        hdr = json.loads(_unb64(head))
        claims = json.loads(_unb64(body))
    except Exception as e:  # noqa: BLE001
        raise PermissionError(f"malformed token: {e}") from None
    if hdr.get("alg") != "HS256":
        raise PermissionError("unsupported token algorithm")
    want = hmac.new(_signing_key(), f"{head}.{body}".encode(), hashlib.sha256).digest()
    if not hmac.compare_digest(want, _unb64(sig)):
        raise PermissionError("bad token signature")
    if claims.get("iss") != ISSUER:
        raise PermissionError("bad token issuer")
    if int(claims.get("exp", 0)) < time.time():
        raise PermissionError("token expired")
    return claims


def password_grant(username: str, password: str, ttl: int = 3600) -> dict:
    """OIDC token-endpoint response for the resource-owner password grant."""
    u = load_users().get(username)
    if u is None or not check_password(password, u.get("hash", "")):
        raise PermissionError("invalid credentials")
    tok = issue_token(u["email"], ttl, u.get("groups"))
    return {"access_token": tok, "id_token": tok, "token_type": "Bearer", "expires_in": int(ttl)}


def discovery(base_url: str) -> dict:
    return {"issuer": ISSUER, "token_endpoint": base_url + "/auth/token",
            "userinfo_endpoint": base_url + "/auth/userinfo", "grant_types_supported": ["password"],
            "id_token_signing_alg_values_supported": ["HS256"], "claims_supported": ["sub", "email", "groups"]}


# ------------------------------------------------------------------------------- certificates
def certs_dir() -> str:
    from ..runtime.storage import mxtrain_home
    return os.path.join(mxtrain_home(), "certs")


def _openssl(*args: str) -> None:
    subprocess.run(["openssl", *args], check=True, capture_output=True)


def _not_after(cert: str) -> float:
    out = subprocess.run(["openssl", "x509", "-in", cert, "-noout", "-enddate"], check=True, capture_output=True,
                         text=True).stdout.strip()
    import email.utils
    return email.utils.parsedate_to_datetime(out.split("=", 1)[1].replace("GMT", "+0000")).timestamp()


def ensure_ca(days: int = 3650) -> Dict[str, str]:
    d = certs_dir()
    os.makedirs(d, exist_ok=True)
    key, crt = os.path.join(d, "ca.key"), os.path.join(d, "ca.crt")
    if not (os.path.exists(key) and os.path.exists(crt)):
        _openssl("req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes",
                 "-keyout", key, "-out", crt, "-days", str(days), "-subj", "/CN=mxtrain-node-ca")
        os.chmod(key, 0o600)
    return {"key": key, "cert": crt}


def issue_cert(name: str, dns: List[str], ips: Optional[List[str]] = None, days: int = 90,
               renew_days: int = 30) -> Dict[str, str]:
    """Server certificate ``name`` signed by the node CA (Certificate + Issuer of
    cert-manager); re-issued when missing or within ``renew_days`` of expiry.  Returns
    {cert, key, ca, renewed}."""
    from ..launch.release import check_name
    check_name(name, "certificate name")
    ca = ensure_ca()
    d = certs_dir()
    key, crt, csr = (os.path.join(d, f"{name}.{x}") for x in ("key", "crt", "csr"))
    if os.path.exists(crt) and os.path.exists(key) and _not_after(crt) - time.time() > renew_days * 86400:
        return {"cert": crt, "key": key, "ca": ca["cert"], "renewed": "no"}
    san = ",".join([f"DNS:{x}" for x in dns] + [f"IP:{x}" for x in (ips or [])])
    ext = os.path.join(d, f"{name}.ext")
    with open(ext, "w") as f:
        f.write(f"subjectAltName={san}\nextendedKeyUsage=serverAuth\n")
    _openssl("req", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes", "-keyout", key,
             "-out", csr, "-subj", f"/CN={dns[0] if dns else name}")
    os.chmod(key, 0o600)
    _openssl("x509", "-req", "-in", csr, "-CA", ca["cert"], "-CAkey", ca["key"], "-CAcreateserial", "-out", crt,
             "-days", str(days), "-extfile", ext)
    for p in (csr, ext):
        os.unlink(p)
    return {"cert": crt, "key": key, "ca": ca["cert"], "renewed": "yes"}


def main(argv=None) -> int:
    """mxtrain identity: add-user EMAIL [--groups g1,g2] (password on stdin) | token EMAIL
    | issue-cert NAME --dns a,b [--ip x]"""
    import argparse
    import sys
    ap = argparse.ArgumentParser(prog="mxtrain identity")
    sub = ap.add_subparsers(dest="cmd", required=True)
    a1 = sub.add_parser("add-user")
    a1.add_argument("email")
    a1.add_argument("--groups", default="")
    a2 = sub.add_parser("issue-cert")
    a2.add_argument("name")
    a2.add_argument("--dns", default="localhost")
    a2.add_argument("--ip", default="")
    a2.add_argument("--days", type=int, default=90)
    a = ap.parse_args(argv)
    if a.cmd == "add-user":
        pw = sys.stdin.readline().rstrip("\n")
        if not pw:
            print("password expected on stdin", file=sys.stderr)
            return 2
        print(json.dumps(add_user(a.email, pw, [g for g in a.groups.split(",") if g])))
        return 0
    c = issue_cert(a.name, [x for x in a.dns.split(",") if x], [x for x in a.ip.split(",") if x], a.days)
    print(json.dumps(c))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

"""L1 side of the AIUS token: ``L1Token`` and the Arbitrum custom-gateway flow it plugs into.

Behavioural twin of ``contract/contracts/L1Token.sol`` plus minimal stand-ins for
the Arbitrum ``L1CustomGateway`` / ``L2GatewayRouter`` it calls, so the deploy sequence of
``contract/scripts/000-deployl1.ts`` -> ``001-deployl2.ts`` -> ``002-register-gateway.ts`` and a
deposit / withdrawal round trip can be replayed in-process against ``MockBaseToken`` (the L2 token,
``bridgeMint``/``bridgeBurn`` restricted to the L2 gateway, BaseTokenV1.sol:53-68):

* ``L1Token`` (L1Token.sol:34-111): OZ ERC20 "Arbius"/"AIUS", Ownable, the whole initial supply
  (in whole tokens, scaled by 10**decimals) preminted to the deployer (:41-49);
  ``isArbitrumEnabled`` answers 0xb1 only while ``registerTokenOnL2`` is running and reverts
  ``NOT_EXPECTED_CALL`` otherwise (:52-55); ``registerTokenOnL2`` is onlyOwner and registers the
  L2 address with the custom gateway, then the gateway with the router (:58-90).
* ``MockL1CustomGateway``: ``registerTokenToL2`` asks the token ``isArbitrumEnabled`` (the callback
  the real gateway makes, which is why the token flips its flag) and records the L1->L2 mapping;
  ``outboundTransfer`` escrows L1 tokens and (as the retryable ticket would) mints on L2 through
  the L2 gateway address; ``finalizeInboundTransfer`` releases escrow after an L2 ``bridgeBurn``.
* ``MockL2GatewayRouter``: ``setGateway`` records token -> gateway (also checks
  ``isArbitrumEnabled``).

Cross-chain messaging is synchronous here (no retryable-ticket delay, no gas accounting): enough
to exercise the token-side invariants (supply conservation across the two chains, gateway-only
mint/burn, owner-only registration), which is what the node and its tests depend on.
"""
from __future__ import annotations

from typing import Dict, Optional

from .mock_engine import MockToken, Revert, ZERO, _addr


class L1Token(MockToken):
    """L1Token.sol:34-111."""

    DECIMALS = 18

    def __init__(self, deployer: str, custom_gateway: "MockL1CustomGateway", router: "MockL2GatewayRouter",
                 initial_supply: int = 1_000_000, address: str = "0x" + "a1" * 20):
        super().__init__("Arbius", "AIUS")
        self.address = _addr(address)
        self.owner = _addr(deployer)
        self.custom_gateway = custom_gateway
        self.router = router
        self._should_register_gateway = False
        self.mint(deployer, initial_supply * 10 ** self.DECIMALS)

    def is_arbitrum_enabled(self) -> int:
        if not self._should_register_gateway:
            raise Revert("NOT_EXPECTED_CALL")
        return 0xB1

    def register_token_on_l2(self, sender: str, l2_custom_token: str, max_submission_cost_gateway: int = 0,
                             max_submission_cost_router: int = 0, max_gas_gateway: int = 0,
                             max_gas_router: int = 0, gas_price_bid: int = 0, value_gateway: int = 0,
                             value_router: int = 0, credit_back: str = ZERO):
        if _addr(sender) != self.owner:
            raise Revert("Ownable: caller is not the owner")
        prev = self._should_register_gateway
        self._should_register_gateway = True
        try:
            self.custom_gateway.register_token_to_l2(self, l2_custom_token)
            self.router.set_gateway(self, self.custom_gateway)
        finally:
            self._should_register_gateway = prev

    def transfer_ownership(self, sender: str, new_owner: str):
        if _addr(sender) != self.owner:
            raise Revert("Ownable: caller is not the owner")
        if _addr(new_owner) == ZERO:
            raise Revert("Ownable: new owner is the zero address")
        self.owner = _addr(new_owner)


class MockL2GatewayRouter:
    def __init__(self, address: str = "0x" + "a2" * 20):
        self.address = _addr(address)
        self.gateways: Dict[str, str] = {}

    def set_gateway(self, token: L1Token, gateway: "MockL1CustomGateway"):
        if token.is_arbitrum_enabled() != 0xB1:          # the router's own callback check
            raise Revert("NOT_ARB_ENABLED")
        self.gateways[token.address] = gateway.address

    def get_gateway(self, token_address: str) -> str:
        return self.gateways.get(_addr(token_address), ZERO)


class MockL1CustomGateway:
    """Escrowing L1 custom gateway + the L2 counterpart's mint/burn, synchronously."""

    def __init__(self, l2_gateway_address: str, address: str = "0x" + "a3" * 20):
        self.address = _addr(address)
        self.l2_gateway_address = _addr(l2_gateway_address)
        self.l1_to_l2: Dict[str, str] = {}
        self.l2_tokens: Dict[str, object] = {}

    def register_token_to_l2(self, token: L1Token, l2_address: str):
        if token.is_arbitrum_enabled() != 0xB1:
            raise Revert("NOT_ARB_ENABLED")
        prev = self.l1_to_l2.get(token.address)
        if prev is not None and prev != _addr(l2_address):
            raise Revert("NO_UPDATE_TO_DIFFERENT_ADDR")
        self.l1_to_l2[token.address] = _addr(l2_address)

    def attach_l2_token(self, l1_token: L1Token, l2_token) -> None:
        """Bind the registered L2 address to its in-process MockBaseToken."""
        if self.l1_to_l2.get(l1_token.address) != _addr(l2_token.address):
            raise Revert("token not registered")
        self.l2_tokens[l1_token.address] = l2_token

    def outbound_transfer(self, sender: str, l1_token: L1Token, to: str, amount: int):
        """Deposit: escrow on L1, mint to ``to`` on L2 (the retryable's finalizeInboundTransfer)."""
        l2 = self.l2_tokens.get(l1_token.address)
        if l2 is None:
            raise Revert("NOT_REGISTERED")
        l1_token.transfer_from(self.address, sender, self.address, amount)
        l2.bridge_mint(self.l2_gateway_address, to, amount)

    def withdraw(self, sender: str, l1_token: L1Token, to: str, amount: int):
        """Withdrawal: burn on L2 through the L2 gateway, release the L1 escrow to ``to``."""
        l2 = self.l2_tokens.get(l1_token.address)
        if l2 is None:
            raise Revert("NOT_REGISTERED")
        l2.bridge_burn(self.l2_gateway_address, sender, amount)
        l1_token.transfer(self.address, to, amount)


def deploy_bridge(deployer: str, l2_token, initial_supply: int = 1_000_000,
                  l2_gateway_address: Optional[str] = None):
    """000-deployl1 + 002-register-gateway against an existing L2 MockBaseToken.

    The L2 token's ``l2_gateway`` must be the gateway address used here (its bridge functions are
    gated on it), so by default the L2 token's configured gateway is reused."""
    l2_gw = _addr(l2_gateway_address or l2_token.l2_gateway)
    gateway = MockL1CustomGateway(l2_gw)
    router = MockL2GatewayRouter()
    token = L1Token(deployer, gateway, router, initial_supply)
    token.register_token_on_l2(deployer, l2_token.address)
    gateway.attach_l2_token(token, l2_token)
    return token, gateway, router

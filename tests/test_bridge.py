"""L1Token + custom-gateway twin (contract/contracts/L1Token.sol, scripts/000-002)."""
import pytest

from arbius_amd.chain.mock_bridge import L1Token, MockL1CustomGateway, MockL2GatewayRouter, deploy_bridge
from arbius_amd.chain.mock_engine import Revert
from arbius_amd.chain.mock_governance import MockBaseToken

E18 = 10 ** 18
DEPLOYER = "0x" + "d1" * 20
ALICE = "0x" + "a0" * 20
L2_GW = "0x" + "9a" * 20


def _setup():
    l2 = MockBaseToken(l2_gateway=L2_GW)
    l1, gw, router = deploy_bridge(DEPLOYER, l2)
    return l1, gw, router, l2


def test_premint_and_metadata():
    gw, router = MockL1CustomGateway(L2_GW), MockL2GatewayRouter()
    t = L1Token(DEPLOYER, gw, router, 1_000_000)
    assert (t.name, t.symbol) == ("Arbius", "AIUS")
    assert t.total_supply == 1_000_000 * E18 == t.balance_of(DEPLOYER)


def test_is_arbitrum_enabled_only_during_registration():
    l1, gw, router, l2 = _setup()
    with pytest.raises(Revert, match="NOT_EXPECTED_CALL"):
        l1.is_arbitrum_enabled()
    assert gw.l1_to_l2[l1.address] == l2.address
    assert router.get_gateway(l1.address) == gw.address


def test_register_only_owner_and_no_address_change():
    gw, router = MockL1CustomGateway(L2_GW), MockL2GatewayRouter()
    t = L1Token(DEPLOYER, gw, router)
    with pytest.raises(Revert, match="Ownable"):
        t.register_token_on_l2(ALICE, "0x" + "bb" * 20)
    t.register_token_on_l2(DEPLOYER, "0x" + "bb" * 20)
    t.register_token_on_l2(DEPLOYER, "0x" + "bb" * 20)            # idempotent
    with pytest.raises(Revert, match="NO_UPDATE_TO_DIFFERENT_ADDR"):
        t.register_token_on_l2(DEPLOYER, "0x" + "cc" * 20)


def test_deposit_and_withdraw_conserve_supply():
    l1, gw, _, l2 = _setup()
    l1.transfer(DEPLOYER, ALICE, 1000 * E18)
    l1.approve(ALICE, gw.address, 2 ** 256 - 1)
    gw.outbound_transfer(ALICE, l1, ALICE, 400 * E18)
    assert l1.balance_of(ALICE) == 600 * E18 and l1.balance_of(gw.address) == 400 * E18
    assert l2.balance_of(ALICE) == 400 * E18 and l2.total_supply == 400 * E18
    gw.withdraw(ALICE, l1, ALICE, 150 * E18)
    assert l2.balance_of(ALICE) == 250 * E18 and l2.total_supply == 250 * E18
    assert l1.balance_of(ALICE) == 750 * E18
    # escrow on L1 always backs the L2 supply
    assert l1.balance_of(gw.address) == l2.total_supply
    with pytest.raises(Revert):
        gw.withdraw(ALICE, l1, ALICE, 10_000 * E18)                # more than bridged


def test_l2_mint_is_gateway_only():
    _, _, _, l2 = _setup()
    with pytest.raises(Revert, match="NOT_GATEWAY"):
        l2.bridge_mint(ALICE, ALICE, 1)

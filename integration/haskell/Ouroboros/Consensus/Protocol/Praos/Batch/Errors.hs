{-# LANGUAGE DataKinds           #-}
{-# LANGUAGE NamedFieldPuns      #-}
{-# LANGUAGE ScopedTypeVariables #-}
{-# LANGUAGE TypeApplications    #-}

-- | The reference's own error values, rebuilt from a batch verdict
-- ('Ouroboros.Consensus.Protocol.Praos.Batch').
--
-- The GPU reports one check bit per predicate and the host fold applies the
-- reference's first-error order (Praos.hs:441-459, @(?!)@ :690-699); the verdict names
-- the first failing predicate.  This module turns it back into the exact constructor,
-- with the payload 'validateKESSignature' (Praos.hs:558-606), 'validateVRFSignature'
-- (:528-556) and the envelope checks (HeaderValidation.hs:297-344,
-- Shelley/Protocol/Praos.hs:66-80) build from the same inputs, so a caller that
-- compares errors (tests, ChainSel tracing) sees what the sequential path would have
-- thrown.  Shipped as source (no GHC where this repository is built); the verdict codes
-- are the PRAOS_V_* values of include/praos_hip.h.
module Ouroboros.Consensus.Protocol.Praos.Batch.Errors
  ( verdictToPraosValidationErr
  , verdictToPraosEnvelopeError
  , verdictToHeaderEnvelopeError
  , TPraosFailure (..)
  , tpraosFailures
  , TPraosOverlaySlot (..)
  , tpraosChainTransitionError
  , verdictToChainPredicateFailure
  ) where

import           Cardano.Crypto.VRF (CertifiedVRF (certifiedOutput), getOutputVRFNatural, hashVerKeyVRF)
import           Cardano.Ledger.BaseTypes (ActiveSlotCoeff, Nonce)
import           Cardano.Ledger.Binary (Version)
import           Cardano.Ledger.Chain (ChainPredicateFailure (..))
import           Cardano.Ledger.Keys (GenDelegPair (..), KeyHash, KeyRole (BlockIssuer, GenesisDelegate), coerceKeyRole,
                     hashKey)
import           Cardano.Ledger.PoolDistr (IndividualPoolStake (..))
import qualified Cardano.Ledger.Shelley.API as SL
import qualified Cardano.Protocol.TPraos.API as TP
import           Cardano.Protocol.TPraos.BHeader (BHBody (..), BHeader (..), BoundedNatural (bvValue), seedEta, seedL)
import           Cardano.Protocol.TPraos.OCert (KESPeriod (..), OCert (..))
import           Cardano.Protocol.TPraos.Rules.OCert (OcertPredicateFailure (..))
import           Cardano.Protocol.TPraos.Rules.Overlay (OverlayPredicateFailure (..))
import           Cardano.Protocol.TPraos.Rules.Prtcl (PrtclPredicateFailure (..))
import           Data.Coerce (coerce)
import           Cardano.Slotting.Block (BlockNo)
import           Cardano.Slotting.Slot (SlotNo (..), WithOrigin)
import           Data.Bits (testBit, (.&.))
import           Data.Map.Strict (Map)
import qualified Data.Map.Strict as Map
import           Data.Maybe (fromMaybe)
import           Data.Proxy (Proxy (..))
import           Data.Word (Word16, Word64, Word8)
import           Numeric.Natural (Natural)
import           Ouroboros.Consensus.Block (ChainHash, HeaderHash)
import           Ouroboros.Consensus.HeaderValidation (HeaderEnvelopeError (..),
                     OtherHeaderEnvelopeError)
import           Ouroboros.Consensus.Protocol.Praos (PraosCrypto, PraosParams (..),
                     PraosValidationErr (..))
import qualified Ouroboros.Consensus.Protocol.Praos.Views as Views
import           Ouroboros.Consensus.Protocol.Praos.VRF (vrfLeaderValue)
import           Ouroboros.Consensus.Shelley.Protocol.Praos (PraosEnvelopeError (..))

-- | A protocol verdict (PRAOS_V_KES_BEFORE_START .. PRAOS_V_LEADER_TOO_BIG = 1..11) as
-- the 'PraosValidationErr' the reference throws for that header.
--
--   * @counters@: the OCert counter map of the state the fold judged the header against
--     (the batch's returned PraosState CBOR up to the header, or one's own fold);
--   * @bits@: the header's check bits, which tell the two KES failure messages apart
--     (Merkle path: Sum KES "Reject"; leaf Ed25519: libsodium "Verification failed").
verdictToPraosValidationErr
  :: forall c. PraosCrypto c
  => PraosParams
  -> ActiveSlotCoeff                          -- ^ praosLeaderF
  -> Nonce                                    -- ^ the ticked epoch nonce
  -> Views.LedgerView c
  -> Map (KeyHash 'BlockIssuer c) Word64      -- ^ OCert counters before the header
  -> Views.HeaderView c
  -> Word8                                    -- ^ verdict (PRAOS_V_*)
  -> Word16                                   -- ^ check bits (PRAOS_BIT_*)
  -> Maybe (PraosValidationErr c)
verdictToPraosValidationErr PraosParams {praosMaxKESEvo, praosSlotsPerKESPeriod} f eta0
                            Views.LedgerView {Views.lvPoolDistr} counters b v bits =
  case v of
    1  -> Just (KESBeforeStartOCERT c0 kp)                          -- Praos.hs:567
    2  -> Just (KESAfterEndOCERT kp c0 praosMaxKESEvo)               -- :568
    3  -> Just (InvalidSignatureOCERT n c0 "Verification failed")    -- :580
    4  -> Just (InvalidKesSignatureOCERT kp_ c0_ t kesMsg)           -- :582
    5  -> Just (NoCounterForKeyHashOCERT hk)                         -- :586-587
    6  -> Just (CounterTooSmallOCERT m n)                            -- :589
    7  -> Just (CounterOverIncrementedOCERT m n)                     -- :590
    8  -> Just (VRFKeyUnknown poolHk)                                -- :536-537
    9  -> (\(vrfHK, _) -> VRFKeyWrongVRFKey poolHk vrfHK (hashVerKeyVRF vrfK)) <$> registered
    10 -> Just (VRFKeyBadProof slot eta0 vrfCert)                    -- :543-547
    11 -> (\(_, sigma) -> VRFLeaderValueTooBig (bvValue (vrfLeaderValue (Proxy @c) vrfCert)) sigma f)
            <$> registered                                           -- :549-550
    _  -> Nothing
  where
    oc = Views.hvOCert b
    OCert _ n c0@(KESPeriod c0_) _ = oc
    SlotNo s = Views.hvSlotNo b
    slot = Views.hvSlotNo b
    kp_ = fromIntegral (s `div` praosSlotsPerKESPeriod)
    kp = KESPeriod kp_
    t = if kp_ >= c0_ then kp_ - c0_ else 0
    kesMsg = if testBit bits 3 then "Reject" else "Verification failed"
    hk = hashKey (Views.hvVK b)
    poolHk = coerceKeyRole hk
    vrfK = Views.hvVrfVK b
    vrfCert = Views.hvVrfRes b
    pd = SL.unPoolDistr lvPoolDistr
    registered = (\(IndividualPoolStake sigma vrfHK) -> (vrfHK, sigma)) <$> Map.lookup poolHk pd
    -- currentIssueNo (Praos.hs:601-606): the counter map, else 0 for a registered pool
    m = fromMaybe 0 (Map.lookup hk counters)

-- | An envelope verdict of the Praos-specific checks (PRAOS_V_ENV_OBSOLETE_NODE,
-- _HEADER_SIZE, _BLOCK_SIZE = 16..18) as 'PraosEnvelopeError'
-- (Shelley/Protocol/Praos.hs:66-80): the caller passes the values envelopeChecks reads
-- (the header's protocol version major and praosMaxMajorPV as 'Version's, the sizes and
-- the ledger view's limits).
verdictToPraosEnvelopeError
  :: (Version, Version)        -- ^ (pvMajor lvProtocolVersion, praosMaxMajorPV)
  -> (Natural, Natural)        -- ^ (header size, lvMaxHeaderSize)
  -> (Natural, Natural)        -- ^ (hbBodySize, lvMaxBodySize)
  -> Word8
  -> Maybe PraosEnvelopeError
verdictToPraosEnvelopeError (m, maxpv) (hs, maxHS) (bs, maxBS) v = case v of
  16 -> Just (ObsoleteNode m maxpv)
  17 -> Just (HeaderSizeTooLarge hs maxHS)
  18 -> Just (BlockSizeTooLarge bs maxBS)
  _  -> Nothing

-- | The generic envelope verdicts (PRAOS_V_ENV_BLOCK_NO, _SLOT_NO, _PREV_HASH = 13..15) as
-- 'HeaderEnvelopeError' (HeaderValidation.hs:213-231), from what validateEnvelope
-- compares (:303-311): the expected and actual block number, the minimum and actual slot,
-- and the tip hash against the header's prev hash; the Praos-specific ones go through
-- 'verdictToPraosEnvelopeError' and 'OtherHeaderEnvelopeError'.
verdictToHeaderEnvelopeError
  :: (BlockNo, BlockNo)
  -> (SlotNo, SlotNo)
  -> (WithOrigin (HeaderHash blk), ChainHash blk)
  -> Maybe (OtherHeaderEnvelopeError blk)
  -> Word8
  -> Maybe (HeaderEnvelopeError blk)
verdictToHeaderEnvelopeError (expB, actB) (expS, actS) (tipH, prevH) other v = case v of
  13 -> Just (UnexpectedBlockNo expB actB)
  14 -> Just (UnexpectedSlotNo expS actS)
  15 -> Just (UnexpectedPrevHash tipH prevH)
  _  | v >= 16 && v <= 18 -> OtherHeaderEnvelopeError <$> other
     | otherwise -> Nothing

-- | The TPraos PRTCL predicate failures of one header (PRAOS_TPF_* bits of
-- praos_tpraos_update_chain_dep_state), named after cardano-protocol-tpraos's
-- OVERLAY / OCERT predicate-failure constructors (ValidateAll collects every OCERT
-- failure and the first of OVERLAY's Either-chain).  'tpraosChainTransitionError' builds
-- the ledger's own 'SL.ChainTransitionError' value from them.
data TPraosFailure
  = TPKESBeforeStartOCERT | TPKESAfterEndOCERT | TPInvalidSignatureOCERT | TPInvalidKesSignatureOCERT
  | TPNoCounterForKeyHashOCERT | TPCounterTooSmallOCERT | TPCounterOverIncrementedOCERT
  | TPVRFKeyUnknown | TPVRFKeyWrongVRFKey | TPVRFKeyBadNonce | TPVRFKeyBadLeaderValue
  | TPVRFLeaderValueTooBig | TPNotActiveSlotOVERLAY | TPWrongGenesisColdKeyOVERLAY
  | TPWrongGenesisVRFKeyOVERLAY
  deriving (Eq, Show, Enum, Bounded)

-- | The failures of a set, in the order ValidateAll collects them (overlayTransition: its own
-- predicates, NotActiveSlot or WrongGenesisColdKey then the first failure of the VRF checks;
-- then the OCERT sub-rule's, in the order ocertTransition checks them).  Mirrored by
-- integration/c/ffi_harness.c TPF_NAMES (tests/test_abi.py checks the two tables agree).
tpraosFailures :: Word16 -> [TPraosFailure]
tpraosFailures f = [x | (bit, x) <- tpraosFailureTable, f .&. bit /= 0]

tpraosFailureTable :: [(Word16, TPraosFailure)]
tpraosFailureTable =
  [ (0x2000, TPNotActiveSlotOVERLAY)          -- PRAOS_TPF_NOT_ACTIVE
  , (0x4000, TPWrongGenesisColdKeyOVERLAY)    -- PRAOS_TPF_GEN_COLD
  , (0x0100, TPVRFKeyUnknown)                 -- PRAOS_TPF_VRF_KEY_UNKNOWN
  , (0x0200, TPVRFKeyWrongVRFKey)             -- PRAOS_TPF_VRF_KEY_WRONG
  , (0x8000, TPWrongGenesisVRFKeyOVERLAY)     -- PRAOS_TPF_GEN_VRF
  , (0x0400, TPVRFKeyBadNonce)                -- PRAOS_TPF_BAD_NONCE
  , (0x0800, TPVRFKeyBadLeaderValue)          -- PRAOS_TPF_BAD_LEADER
  , (0x1000, TPVRFLeaderValueTooBig)          -- PRAOS_TPF_LEADER_TOO_BIG
  , (0x0001, TPKESBeforeStartOCERT)           -- PRAOS_TPF_KES_BEFORE_START
  , (0x0002, TPKESAfterEndOCERT)              -- PRAOS_TPF_KES_AFTER_END
  , (0x0004, TPInvalidSignatureOCERT)         -- PRAOS_TPF_OCERT_SIG
  , (0x0008, TPInvalidKesSignatureOCERT)      -- PRAOS_TPF_KES_SIG
  , (0x0010, TPNoCounterForKeyHashOCERT)      -- PRAOS_TPF_COUNTER_MISSING
  , (0x0020, TPCounterTooSmallOCERT)          -- PRAOS_TPF_COUNTER_TOO_SMALL
  , (0x0040, TPCounterOverIncrementedOCERT)   -- PRAOS_TPF_COUNTER_OVER_INC
  ]

-- | What the overlay schedule says about the header's slot (lookupInOverlaySchedule of
-- cardano-protocol-tpraos Rules/Overlay.hs, which the caller runs over the ledger view's
-- genesis keys and decentralisation parameter): a Praos slot, a non-active overlay slot, or an
-- active one with the scheduled genesis key's delegation pair.
data TPraosOverlaySlot c
  = TPraosSlot
  | TPraosNonActiveSlot
  | TPraosActiveSlot !(GenDelegPair c)

-- | A TPraos header's PRTCL failure set as the reference's error, 'SL.ChainTransitionError'
-- (ValidationErr (TPraos c), TPraos.hs:299; thrown by SL.updateChainDepState, :378-387), every
-- failure with the payload cardano-protocol-tpraos's rules build from the same header,
-- ledger view and state:
--
--   * OVERLAY (Rules/Overlay.hs overlayTransition / praosVrfChecks / pbftVrfChecks / vrfChecks):
--     VRFKeyUnknown hk, VRFKeyWrongVRFKey hk registered (hashVerKeyVRF vrfVk),
--     VRFKeyBadNonce seedEta slot eta0 eta-cert, VRFKeyBadLeaderValue seedL slot eta0 L-cert,
--     VRFLeaderValueTooBig (getOutputVRFNatural L-output) sigma f, NotActiveSlotOVERLAY slot,
--     WrongGenesisColdKeyOVERLAY vkh delegate, WrongGenesisVRFKeyOVERLAY vkh delegate-vrf
--     (hashVerKeyVRF vrfVk);
--   * OCERT (Rules/OCert.hs ocertTransition), under 'OcertFailure': KESBeforeStartOCERT c0 kp,
--     KESAfterEndOCERT kp c0 maxKESEvo, InvalidSignatureOCERT n c0 "Verification failed",
--     InvalidKesSignatureOCERT kp c0 t ("Reject" for the Merkle path, libsodium's
--     "Verification failed" for the leaf: the check bits tell them apart),
--     NoCounterForKeyHashOCERT hk, CounterTooSmallOCERT m n, CounterOverIncrementedOCERT m n.
--
-- Every failure is wrapped as PRTCL's 'OverlayFailure' (UPDN has no failures), in the order
-- 'tpraosFailures' lists them.
tpraosChainTransitionError
  :: forall c. TP.PraosCrypto c
  => Word64                                   -- ^ slotsPerKESPeriod
  -> Word64                                   -- ^ maxKESEvo
  -> ActiveSlotCoeff
  -> TP.LedgerView c
  -> Nonce                                    -- ^ the ticked epoch nonce (ticknStateEpochNonce)
  -> Map (KeyHash 'BlockIssuer c) Word64      -- ^ OCert counters before the header (csCounters)
  -> TPraosOverlaySlot c
  -> BHeader c
  -> Word16                                   -- ^ failure set (PRAOS_TPF_*)
  -> Word16                                   -- ^ check bits (PRAOS_BIT_*)
  -> TP.ChainTransitionError c
tpraosChainTransitionError spkp maxEvo f lv eta0 counters ovl (BHeader bhb _) fails bits =
  TP.ChainTransitionError (map (OverlayFailure . failure) (tpraosFailures fails))
  where
    failure x = case x of
      TPNotActiveSlotOVERLAY       -> NotActiveSlotOVERLAY slot
      TPWrongGenesisColdKeyOVERLAY -> WrongGenesisColdKeyOVERLAY vkh (delegate genDelegKeyHash)
      TPVRFKeyUnknown              -> VRFKeyUnknown poolHk
      TPVRFKeyWrongVRFKey          -> VRFKeyWrongVRFKey poolHk (maybe vrfHdr fst registered) vrfHdr
      TPWrongGenesisVRFKeyOVERLAY  -> WrongGenesisVRFKeyOVERLAY vkh (delegate genDelegVrfHash) vrfHdr
      TPVRFKeyBadNonce             -> VRFKeyBadNonce seedEta slot eta0 (coerce (bheaderEta bhb))
      TPVRFKeyBadLeaderValue       -> VRFKeyBadLeaderValue seedL slot eta0 (coerce (bheaderL bhb))
      TPVRFLeaderValueTooBig       -> VRFLeaderValueTooBig (getOutputVRFNatural (certifiedOutput (bheaderL bhb)))
                                                           (maybe 0 snd registered) f
      TPKESBeforeStartOCERT        -> OcertFailure (KESBeforeStartOCERT c0 kp)
      TPKESAfterEndOCERT           -> OcertFailure (KESAfterEndOCERT kp c0 maxEvo)
      TPInvalidSignatureOCERT      -> OcertFailure (InvalidSignatureOCERT n c0 "Verification failed")
      TPInvalidKesSignatureOCERT   -> OcertFailure (InvalidKesSignatureOCERT kp_ c0_ t kesMsg)
      TPNoCounterForKeyHashOCERT   -> OcertFailure (NoCounterForKeyHashOCERT vkh)
      TPCounterTooSmallOCERT       -> OcertFailure (CounterTooSmallOCERT m n)
      TPCounterOverIncrementedOCERT -> OcertFailure (CounterOverIncrementedOCERT m n)
    slot@(SlotNo s) = bheaderSlotNo bhb
    OCert _ n c0@(KESPeriod c0_) _ = bheaderOCert bhb
    kp_ = fromIntegral (s `div` spkp)
    kp = KESPeriod kp_
    t = if kp_ >= c0_ then kp_ - c0_ else 0
    kesMsg = if testBit bits 3 then "Reject" else "Verification failed"
    vkh = hashKey (bheaderVk bhb) :: KeyHash 'BlockIssuer c
    poolHk = coerceKeyRole vkh
    vrfHdr = hashVerKeyVRF (bheaderVrfVk bhb)
    registered = (\(IndividualPoolStake sigma vrfHK) -> (vrfHK, sigma)) <$>
                 Map.lookup poolHk (SL.unPoolDistr (TP.lvPoolDistr lv))
    delegate :: (GenDelegPair c -> a) -> a
    delegate sel = case ovl of
      TPraosActiveSlot p -> sel p
      _ -> error "tpraosChainTransitionError: a genesis-key failure outside an active overlay slot"
    -- currentIssueNo (Rules/OCert.hs): the counter map, else 0 for a registered pool or a
    -- genesis delegate (NoCounterForKeyHashOCERT otherwise, reported by its own bit)
    m = fromMaybe 0 (Map.lookup vkh counters)

-- | A TPraos envelope verdict of the ledger's chain checks (PRAOS_V_ENV_OBSOLETE_NODE,
-- _HEADER_SIZE, _BLOCK_SIZE = 16..18) as 'ChainPredicateFailure', the EnvelopeCheckError of
-- TPraos (Shelley/Protocol/TPraos.hs: envelopeChecks = SL.chainChecks maxPV lvChainChecks):
-- the protocol version major against MaxMajorProtVer, the header size and the block size
-- against the ledger's limits.
verdictToChainPredicateFailure
  :: (Version, Version)        -- ^ (pvMajor ccProtocolVersion, MaxMajorProtVer)
  -> (Natural, Natural)        -- ^ (header size, ccMaxBHSize)
  -> (Natural, Natural)        -- ^ (bsize, ccMaxBBSize)
  -> Word8
  -> Maybe ChainPredicateFailure
verdictToChainPredicateFailure (m, maxpv) (hs, maxHS) (bs, maxBS) v = case v of
  16 -> Just (ObsoleteNodeCHAIN m maxpv)
  17 -> Just (HeaderSizeTooLargeCHAIN hs maxHS)
  18 -> Just (BlockSizeTooLargeCHAIN bs maxBS)
  _  -> Nothing

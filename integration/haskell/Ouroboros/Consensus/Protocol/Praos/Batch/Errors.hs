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
  ) where

import           Cardano.Crypto.VRF (hashVerKeyVRF)
import           Cardano.Ledger.BaseTypes (ActiveSlotCoeff, Nonce)
import           Cardano.Ledger.Binary (Version)
import           Cardano.Ledger.Keys (KeyHash, KeyRole (BlockIssuer), coerceKeyRole, hashKey)
import           Cardano.Ledger.PoolDistr (IndividualPoolStake (..))
import qualified Cardano.Ledger.Shelley.API as SL
import           Cardano.Protocol.TPraos.BHeader (BoundedNatural (bvValue))
import           Cardano.Protocol.TPraos.OCert (KESPeriod (..), OCert (..))
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
-- failure and the first of OVERLAY's Either-chain).  Building the ledger's own
-- 'SL.ChainTransitionError' values needs the header's views exactly as above; the
-- names and order are what a caller maps onto them.
data TPraosFailure
  = TPKESBeforeStartOCERT | TPKESAfterEndOCERT | TPInvalidSignatureOCERT | TPInvalidKesSignatureOCERT
  | TPNoCounterForKeyHashOCERT | TPCounterTooSmallOCERT | TPCounterOverIncrementedOCERT
  | TPVRFKeyUnknown | TPVRFKeyWrongVRFKey | TPVRFKeyBadNonce | TPVRFKeyBadLeaderValue
  | TPVRFLeaderValueTooBig | TPNotActiveSlotOVERLAY | TPWrongGenesisColdKeyOVERLAY
  | TPWrongGenesisVRFKeyOVERLAY
  deriving (Eq, Show, Enum, Bounded)

tpraosFailures :: Word16 -> [TPraosFailure]
tpraosFailures f = [x | (bit, x) <- table, f .&. bit /= 0]
  where
    table = [ (0x0001, TPKESBeforeStartOCERT), (0x0002, TPKESAfterEndOCERT), (0x0004, TPInvalidSignatureOCERT)
            , (0x0008, TPInvalidKesSignatureOCERT), (0x0010, TPNoCounterForKeyHashOCERT)
            , (0x0020, TPCounterTooSmallOCERT), (0x0040, TPCounterOverIncrementedOCERT)
            , (0x0100, TPVRFKeyUnknown), (0x0200, TPVRFKeyWrongVRFKey), (0x0400, TPVRFKeyBadNonce)
            , (0x0800, TPVRFKeyBadLeaderValue), (0x1000, TPVRFLeaderValueTooBig)
            , (0x2000, TPNotActiveSlotOVERLAY), (0x4000, TPWrongGenesisColdKeyOVERLAY)
            , (0x8000, TPWrongGenesisVRFKeyOVERLAY) ]

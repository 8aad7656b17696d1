{-# LANGUAGE FlexibleContexts    #-}
{-# LANGUAGE NamedFieldPuns      #-}
{-# LANGUAGE RecordWildCards     #-}
{-# LANGUAGE ScopedTypeVariables #-}
{-# LANGUAGE TypeApplications    #-}

-- | 'validateHeader' (ouroboros-consensus HeaderValidation.hs:413-432) folded over the
-- headers of one epoch of a Praos (Babbage / Conway) chain, as one GPU batch.
--
-- The reference validates a chain fragment header by header:
--
-- > foldM (\st hdr -> validateHeader cfg lv hdr (tickHeaderState cfg lv (blockSlot hdr) st)) st0 hdrs
-- >   :: Except (HeaderError blk) (HeaderState blk)
--
-- 'validateEpochHeaders' returns the same value -- the 'HeaderState' after the last header,
-- or the first invalid header's 'HeaderError' together with its index and the state the fold
-- had reached -- and, per header, the batch verdict and check bits as Storable vectors (no
-- boxed list of n cells on the caller's side: an epoch is 432k headers).  The typed error is
-- rebuilt only for the header that stops the fold ('Batch.Errors'), from that one header's
-- views; the other headers are verdict bytes.  'headerOutcome' gives the per-header
-- @Either (HeaderError blk) ()@ view of the same result.
--
-- Foreign calls, in order (replayed from C by integration/c/ffi_harness.c, phase "typed"):
--   praos_ticked_epoch_nonce -> praos_set_epoch -> [praos_host_register of the arena when it
--   is >= 64 MiB] -> praos_verify_header_bytes (decoded fields) -> praos_validate_headers ->
--   praos_state_encode -> [praos_host_unregister].
--
-- Shipped as source (no GHC where this repository is built).
module Ouroboros.Consensus.Protocol.Praos.Batch.Validate
  ( PraosBlockOps (..)
  , EpochHeaders (..)
  , EpochValidation (..)
  , validateEpochHeaders
  , headerOutcome
  , praosParamsC
  , poolDistrEntries
    -- * TPraos (Shelley..Alonzo)
  , TPraosBlockOps (..)
  , EpochValidationTPraos (..)
  , validateEpochHeadersTPraos
  , tpraosToPraosState
  , praosToTPraosState
  ) where

import           Codec.Serialise (Serialise, deserialiseOrFail, serialise)
import           Control.Exception (throwIO)
import           Control.Monad (when)
import qualified Data.ByteString as BS
import qualified Data.ByteString.Lazy as BSL
import           Data.Fixed (Fixed (MkFixed))
import qualified Data.Map.Strict as Map
import           Data.Proxy (Proxy (..))
import qualified Data.Vector.Storable as VS
import qualified Data.Vector.Storable.Mutable as VSM
import           Data.Word (Word16, Word32, Word64, Word8)
import           Numeric.Natural (Natural)

import           Cardano.Crypto.Hash (hashFromBytes, hashToBytes)
import           Cardano.Ledger.BaseTypes (ActiveSlotCoeff, Nonce (..), ProtVer (..), activeSlotLog, activeSlotVal,
                     unboundRational)
import           Cardano.Ledger.Binary (Version, getVersion64)
import           Cardano.Ledger.Keys (KeyHash (..))
import           Cardano.Ledger.PoolDistr (IndividualPoolStake (..), PoolDistr (..))
import           Cardano.Slotting.Slot (WithOrigin (..))
import           Ouroboros.Consensus.Block (BlockProtocol, GetPrevHash (..), HasHeader, Header, HeaderHash,
                     blockNo, blockSlot)
import           Ouroboros.Consensus.HeaderValidation (AnnTip (..), BasicEnvelopeValidation (..),
                     HasAnnTip (..), HeaderError (..), HeaderState (..), OtherHeaderEnvelopeError)
import           Ouroboros.Consensus.Protocol.Abstract (ChainDepState, ValidationErr)
import           Ouroboros.Consensus.Protocol.Praos (PraosParams (..), PraosState (..), PraosValidationErr)
import qualified Ouroboros.Consensus.Protocol.Praos.Views as Views
import           Ouroboros.Consensus.Shelley.Protocol.Praos (PraosEnvelopeError)
import           Ouroboros.Consensus.Protocol.TPraos (TPraosState (..))
import           Cardano.Ledger.Chain (ChainPredicateFailure)
import           Cardano.Ledger.Keys (GenDelegPair (..), GenDelegs (..))
import qualified Cardano.Protocol.TPraos.API as TP
import           Cardano.Protocol.TPraos.BHeader (BHeader)
import qualified Cardano.Protocol.TPraos.Rules.Overlay as Overlay
import qualified Cardano.Protocol.TPraos.Rules.Prtcl as Prtcl
import qualified Cardano.Protocol.TPraos.Rules.Tickn as Tickn
import           Cardano.Slotting.Slot (SlotNo (..))

import           Ouroboros.Consensus.Protocol.Praos.Batch
import           Ouroboros.Consensus.Protocol.Praos.Batch.Errors

-- | The block-specific pieces the fold needs, for a block whose protocol is @Praos c@
-- (ShelleyBlock (Praos c) era: every conversion below is 'id' or a newtype unwrap).
data PraosBlockOps blk c = PraosBlockOps
  { pbView        :: Header blk -> Views.HeaderView c
      -- ^ validateView (configBlock cfg)
  , pbHashBytes   :: HeaderHash blk -> BS.ByteString
      -- ^ the 32 bytes of a header hash (unShelleyHash, hashToBytes)
  , pbSizes       :: Header blk -> (Natural, Natural)
      -- ^ (header size, hbBodySize): what envelopeChecks compares (Shelley/Protocol/Praos.hs:66-80)
  , pbToState     :: ChainDepState (BlockProtocol blk) -> PraosState c
  , pbFromState   :: PraosState c -> ChainDepState (BlockProtocol blk)
  , pbProtocolErr :: PraosValidationErr c -> ValidationErr (BlockProtocol blk)
  , pbEnvelopeErr :: PraosEnvelopeError -> OtherHeaderEnvelopeError blk
  }

-- | One epoch's headers as the ImmutableDB stores them: the header spans back to back in one
-- arena (what 'GetRawHeader' streams), their offsets and lengths, and a way to decode header
-- i (called for the header that stops the fold and for the last valid header's 'AnnTip'), and
-- whether the caller keeps the arena page-locked itself ('PinnedByCaller': an arena reused epoch
-- after epoch, registered once per growth, so no pinning happens inside the call).
data EpochHeaders blk = EpochHeaders
  { ehArena  :: !BS.ByteString
  , ehOffset :: !(VS.Vector Word64)
  , ehLength :: !(VS.Vector Word32)
  , ehDecode :: Int -> Header blk
  , ehPin    :: !ArenaPin
  }

-- | The outcome of the fold and the batch's per-header verdicts (PRAOS_V_*: 0 valid; the
-- first non-zero one stops the fold, later headers carry would-be verdicts) and check bits
-- (PRAOS_BIT_*), unboxed.
data EpochValidation blk = EpochValidation
  { evVerdicts :: !(VS.Vector Word8)
  , evBits     :: !(VS.Vector Word16)
  , evAccepted :: !Int
      -- ^ headers validateHeader accepts before the first invalid one
  , evOutcome  :: !(Either (Int, HeaderError blk, HeaderState blk) (HeaderState blk))
      -- ^ Left: the first invalid header's index, its error and the state before it
  }

-- | What the sequential fold says about header i: @Right ()@ while it is accepted, @Left@ its
-- error at the stop, Nothing after the stop (the reference never reaches those headers).
headerOutcome :: EpochValidation blk -> Int -> Maybe (Either (HeaderError blk) ())
headerOutcome EpochValidation {evAccepted, evOutcome} i
  | i < evAccepted = Just (Right ())
  | otherwise = case evOutcome of
      Left (k, e, _) | k == i -> Just (Left e)
      _                       -> Nothing

-- | PraosParams + the active slot coefficient as the ABI takes them: activeSlotLog f as its
-- Fixed E34 raw integer, f == 1, and the verifyCertified output comparison (True for the
-- cardano-crypto-class >= 2.1 the snapshot pins; see 'PraosParamsC').
praosParamsC :: PraosParams -> ActiveSlotCoeff -> PraosParamsC
praosParamsC PraosParams {praosSlotsPerKESPeriod, praosMaxKESEvo} f =
  PraosParamsC { ppSlotsPerKESPeriod = praosSlotsPerKESPeriod
               , ppMaxKESEvo = praosMaxKESEvo
               , ppFIsOne = unboundRational (activeSlotVal f) == 1
               , ppActiveSlotLogRaw = let MkFixed raw = activeSlotLog f in raw
               , ppVrfCheckOutput = True }

-- | The PoolDistr of a ledger view as (pool key hash, VRF key hash, Fixed E34 raw sigma):
-- sigma = fromRational individualPoolStake, i.e. floor (sigma * 10^34).
poolDistrEntries :: PoolDistr c -> [(BS.ByteString, BS.ByteString, Integer)]
poolDistrEntries (PoolDistr m) =
  [ (hashToBytes kh, hashToBytes vrf, floor (sigma * 10 ^ (34 :: Int)))
  | (KeyHash kh, IndividualPoolStake sigma vrf) <- Map.toList m ]

-- | 'validateHeader' over one epoch's headers (chain order, all in the epoch of the first),
-- from the unticked 'HeaderState' before them and the epoch's ledger view.  The header-state
-- tick (tickHeaderState -> tickChainDepState, Praos.hs:407-431) happens inside the batch fold
-- at each header, as in the reference.
validateEpochHeaders
  :: forall blk c.
     ( BasicEnvelopeValidation blk, HasAnnTip blk, GetPrevHash blk, HasHeader (Header blk)
     , Serialise (PraosState c) )
  => PraosBatchCtx
  -> PraosBlockOps blk c
  -> PraosParams
  -> ActiveSlotCoeff                          -- ^ praosLeaderF
  -> (Word64, Word64, Word64, Word64)         -- ^ epoch layout: base slot, base epoch, length, window
  -> Version                                  -- ^ praosMaxMajorPV
  -> Views.LedgerView c                       -- ^ the epoch's ledger view
  -> HeaderState blk
  -> EpochHeaders blk
  -> IO (EpochValidation blk)
validateEpochHeaders ctx ops pp f ei maxPV lv st0 EpochHeaders {ehArena, ehOffset, ehLength, ehDecode, ehPin} = do
  let n = VS.length ehOffset
  when (VS.length ehLength /= n) $ throwIO (PraosBatchError (-1) "offsets and lengths differ in length")
  if n == 0 then pure (EpochValidation VS.empty VS.empty 0 (Right st0)) else do
    let Views.LedgerView {Views.lvPoolDistr, Views.lvMaxHeaderSize, Views.lvMaxBodySize,
                          Views.lvProtocolVersion = ProtVer pvMajor _} = lv
        stateCbor = BSL.toStrict (serialise (pbToState ops (headerStateChainDep st0)))
        tip0 = case headerStateTip st0 of
          Origin -> Nothing
          NotOrigin t -> Just (fromSlot (annTipSlotNo t), fromBlock (annTipBlockNo t), pbHashBytes ops (annTipHash t))
        limits = (getVersion64 maxPV, getVersion64 pvMajor, fromIntegral lvMaxHeaderSize, fromIntegral lvMaxBodySize)
        firstSlot = fromSlot (blockSlot (ehDecode 0))
    eta <- praosTickedEpochNonce stateCbor ei firstSlot
    praosSetEpoch ctx eta (poolDistrEntries lvPoolDistr) (praosParamsC pp f)
    verdicts <- VSM.new n
    bits <- VSM.new n
    r <- praosValidateHeaderSpans ctx ei limits tip0 stateCbor ehPin ehArena ehOffset ehLength verdicts bits
    vs <- VS.unsafeFreeze verdicts
    bs <- VS.unsafeFreeze bits
    let stop = srChainStop r
        -- the HeaderState after the first k headers: their last one's AnnTip and the
        -- PraosState the batch fold returned (the state at the stop)
        stateAfter k = HeaderState (if k == 0 then headerStateTip st0 else NotOrigin (getAnnTip (ehDecode (k - 1))))
                                   (pbFromState ops (decodeState (srState r)))
    if stop >= n
      then pure (EpochValidation vs bs n (Right (stateAfter n)))
      else do
        let before = stateAfter stop
            -- the epoch nonce the stopping header was judged under is the ticked one
            -- (Praos.hs:454 reads it from the ticked state), which the unticked 'before' does
            -- not carry when the stop is the epoch's first header: pass tickChainDepState's
            err = stopError ops pp f maxPV lv eta before (ehDecode stop) (vs VS.! stop) (bs VS.! stop)
        pure (EpochValidation vs bs stop (Left (stop, err, before)))
  where
    fromSlot s = fromIntegral (fromEnum s) :: Word64
    fromBlock b = fromIntegral (fromEnum b) :: Word64
    decodeState cbor = case deserialiseOrFail (BSL.fromStrict cbor) of
      Right s -> s
      Left e  -> error ("PraosState CBOR returned by the batch fold: " ++ show e)

-- | The HeaderError validateHeader throws for the header that stops the fold: envelope
-- verdicts (PRAOS_V_ENV_*, 13..18) as 'HeaderEnvelopeError' with validateEnvelope's
-- expected values (HeaderValidation.hs:303-345), protocol verdicts (1..11) as
-- 'HeaderProtocolError' rebuilt against the state the fold reached (Batch.Errors).
stopError
  :: forall blk c. (BasicEnvelopeValidation blk, HasAnnTip blk, GetPrevHash blk, HasHeader (Header blk))
  => PraosBlockOps blk c -> PraosParams -> ActiveSlotCoeff -> Version -> Views.LedgerView c
  -> Maybe BS.ByteString -> HeaderState blk -> Header blk -> Word8 -> Word16 -> HeaderError blk
stopError ops pp f maxPV lv eta before hdr v bits
  | v >= 13 && v <= 18 =
      let oldTip = headerStateTip before
          p = Proxy @blk
          expB = case oldTip of
            Origin      -> expectedFirstBlockNo p
            NotOrigin t -> expectedNextBlockNo p (annTipInfo t) (getTipInfo hdr) (annTipBlockNo t)
          expS = case oldTip of
            Origin      -> minimumPossibleSlotNo p
            NotOrigin t -> minimumNextSlotNo p (annTipInfo t) (getTipInfo hdr) (annTipSlotNo t)
          ProtVer pvMajor _ = Views.lvProtocolVersion lv
          (hsize, bsize) = pbSizes ops hdr
          other = pbEnvelopeErr ops <$>
            verdictToPraosEnvelopeError (pvMajor, maxPV) (hsize, Views.lvMaxHeaderSize lv)
                                        (bsize, Views.lvMaxBodySize lv) v
      in maybe (error ("envelope verdict " ++ show v ++ " without its error")) HeaderEnvelopeError $
           verdictToHeaderEnvelopeError (expB, blockNo hdr) (expS, blockSlot hdr)
                                        (annTipHash <$> oldTip, headerPrevHash hdr) other v
  | otherwise =
      -- the OCert counters do not change at a tick: the unticked state's are the ticked ones
      let PraosState {praosStateOCertCounters} = pbToState ops (headerStateChainDep before)
      in maybe (error ("protocol verdict " ++ show v ++ " without its error")) (HeaderProtocolError . pbProtocolErr ops) $
           verdictToPraosValidationErr pp f (toNonce eta) lv praosStateOCertCounters (pbView ops hdr) v bits

-- | A nonce from praos_ticked_epoch_nonce (Nothing = NeutralNonce).
toNonce :: Maybe BS.ByteString -> Nonce
toNonce Nothing = NeutralNonce
toNonce (Just h) = maybe (error "a 32-byte nonce") Nonce (hashFromBytes h)

-- ---------------------------------------------------------------- TPraos (Shelley..Alonzo)

-- | The block-specific pieces for a block whose protocol is @TPraos c@ (ShelleyBlock (TPraos c)
-- era, the eras HFEras.hs:43-49 maps to TPraos): the ValidateView is the header itself
-- (TPraos.hs:151, @SL.BHeader c@), the ValidationErr the ledger's 'TP.ChainTransitionError'
-- (TPraos.hs:299), the envelope's own error the ledger's chain checks
-- (Shelley/Protocol/TPraos.hs envelopeChecks = SL.chainChecks: 'ChainPredicateFailure').
data TPraosBlockOps blk c = TPraosBlockOps
  { tpView        :: Header blk -> BHeader c
  , tpHashBytes   :: HeaderHash blk -> BS.ByteString
  , tpSizes       :: Header blk -> (Natural, Natural)
      -- ^ (bHeaderSize, bsize): what chainChecks compares
  , tpToState     :: ChainDepState (BlockProtocol blk) -> TPraosState c
  , tpFromState   :: TPraosState c -> ChainDepState (BlockProtocol blk)
  , tpProtocolErr :: TP.ChainTransitionError c -> ValidationErr (BlockProtocol blk)
  , tpEnvelopeErr :: ChainPredicateFailure -> OtherHeaderEnvelopeError blk
  }

-- | 'EpochValidation' plus each header's PRTCL failure set (PRAOS_TPF_*, 0 for a valid one).
data EpochValidationTPraos blk = EpochValidationTPraos
  { evtValidation :: !(EpochValidation blk)
  , evtFailures   :: !(VS.Vector Word16)
  }

-- | TPraosState (TPraos.hs:254-257) as the PraosState the ABI's fold reads and writes: the
-- reference's own translation at the Alonzo -> Babbage boundary (Praos/Translate.hs
-- translateChainDepState): counters and the evolving / candidate nonces of PrtclState, the
-- epoch nonce and the previous epoch's last-block nonce of TicknState, the lab nonce.
tpraosToPraosState :: TPraosState c -> PraosState c
tpraosToPraosState (TPraosState lastSlot (TP.ChainDepState (Prtcl.PrtclState counters ev cand) tickn lab)) =
  PraosState { praosStateLastSlot = lastSlot
             , praosStateOCertCounters = counters
             , praosStateEvolvingNonce = ev
             , praosStateCandidateNonce = cand
             , praosStateEpochNonce = Tickn.ticknStateEpochNonce tickn
             , praosStateLabNonce = lab
             , praosStateLastEpochBlockNonce = Tickn.ticknStatePrevHashNonce tickn }

-- | The inverse of 'tpraosToPraosState'.
praosToTPraosState :: PraosState c -> TPraosState c
praosToTPraosState PraosState {..} =
  TPraosState praosStateLastSlot $
    TP.ChainDepState (Prtcl.PrtclState praosStateOCertCounters praosStateEvolvingNonce praosStateCandidateNonce)
                     (Tickn.TicknState praosStateEpochNonce praosStateLastEpochBlockNonce)
                     praosStateLabNonce

-- | 'validateHeader' over one epoch of a TPraos chain, as one GPU batch (on one device or a
-- group: 'withPraosBatchDevices'): the same fold as 'validateEpochHeaders' with TPraos's
-- rules -- TICKN with the ledger view's extra entropy, the two VRF certificates and the 2^512
-- leader bound, the decentralisation overlay when d > 0 (praos_set_overlay), every OCERT
-- predicate collected -- returning the 'HeaderState' after the last header or the first
-- invalid header's 'HeaderError', whose protocol part is the ledger's
-- 'TP.ChainTransitionError' rebuilt with every predicate failure's payload
-- ('tpraosChainTransitionError').
--
-- Foreign calls, in order (integration/c/ffi_harness.c phases "binding" / "binding_group" with
-- a TPraos database): praos_tpraos_ticked_epoch_nonce -> praos_[group_]set_epoch ->
-- [praos_[group_]set_overlay] -> [praos_[group_]host_register] ->
-- praos_[group_]verify_tpraos_header_bytes -> [unregister] -> praos_tpraos_update_chain_dep_state
-- (member 0) -> praos_state_encode.
validateEpochHeadersTPraos
  :: forall blk c.
     ( BasicEnvelopeValidation blk, HasAnnTip blk, GetPrevHash blk, HasHeader (Header blk)
     , Serialise (PraosState c), TP.PraosCrypto c )
  => PraosBatchCtx
  -> TPraosBlockOps blk c
  -> (Word64, Word64, ActiveSlotCoeff)        -- ^ slotsPerKESPeriod, maxKESEvo, activeSlotCoeff (Globals)
  -> Integer                                  -- ^ activeSlotLog f as its Fixed E34 raw integer
  -> (Word64, Word64, Word64, Word64)         -- ^ epoch layout: base slot, base epoch, length, window
  -> Version                                  -- ^ MaxMajorProtVer
  -> TP.LedgerView c                          -- ^ the epoch's ledger view
  -> HeaderState blk
  -> EpochHeaders blk
  -> IO (EpochValidationTPraos blk)
validateEpochHeadersTPraos ctx ops (spkp, maxEvo, f) cRaw ei@(baseSlot, _, epochLen, _) maxPV lv st0
                           EpochHeaders {ehArena, ehOffset, ehLength, ehDecode, ehPin} = do
  let n = VS.length ehOffset
  when (VS.length ehLength /= n) $ throwIO (PraosBatchError (-1) "offsets and lengths differ in length")
  if n == 0 then pure (EpochValidationTPraos (EpochValidation VS.empty VS.empty 0 (Right st0)) VS.empty) else do
    let TP.LedgerView {TP.lvD, TP.lvExtraEntropy, TP.lvPoolDistr, TP.lvGenDelegs = GenDelegs dms,
                       TP.lvChainChecks = TP.ChainChecksPParams {TP.ccMaxBHSize, TP.ccMaxBBSize,
                                                                 TP.ccProtocolVersion = ProtVer pvMajor _}} = lv
        stateCbor = BSL.toStrict (serialise (tpraosToPraosState (tpToState ops (headerStateChainDep st0))))
        tip0 = case headerStateTip st0 of
          Origin -> Nothing
          NotOrigin t -> Just (fromSlot (annTipSlotNo t), fromBlock (annTipBlockNo t), tpHashBytes ops (annTipHash t))
        limits = (getVersion64 maxPV, getVersion64 pvMajor, fromIntegral ccMaxBHSize, fromIntegral ccMaxBBSize)
        firstSlot = fromSlot (blockSlot (ehDecode 0))
        extra = nonceBytes lvExtraEntropy
        pp = PraosParamsC { ppSlotsPerKESPeriod = spkp, ppMaxKESEvo = maxEvo
                          , ppFIsOne = unboundRational (activeSlotVal f) == 1
                          , ppActiveSlotLogRaw = cRaw, ppVrfCheckOutput = True }
        d = unboundRational lvD
    eta <- praosTickedEpochNonceTPraos stateCbor ei firstSlot extra
    praosSetEpoch ctx eta (poolDistrEntries lvPoolDistr) pp
    -- (with d = 0 too: the genesis delegates stay known issuers for OCERT's currentIssueNo)
    praosSetOverlay ctx $ if Map.null dms then Nothing else Just OverlayC
      { ovD = d, ovF = unboundRational (activeSlotVal f), ovEpochBase = baseSlot, ovEpochLength = epochLen
      , ovGenDelegs = [ (hashToBytes g, hashToBytes dk, hashToBytes vrf)
                      | (KeyHash g, GenDelegPair (KeyHash dk) vrf) <- Map.toList dms ] }
    verdicts <- VSM.new n
    fails <- VSM.new n
    bits <- VSM.new n
    r <- praosValidateTPraosHeaderSpans ctx ei limits extra tip0 stateCbor ehPin ehArena ehOffset ehLength verdicts fails
                                        bits
    vs <- VS.unsafeFreeze verdicts
    fs <- VS.unsafeFreeze fails
    bs <- VS.unsafeFreeze bits
    let stop = srChainStop r
        stateAfter k = HeaderState (if k == 0 then headerStateTip st0 else NotOrigin (getAnnTip (ehDecode (k - 1))))
                                   (tpFromState ops (praosToTPraosState (decodeState (srState r))))
    if stop >= n
      then pure (EpochValidationTPraos (EpochValidation vs bs n (Right (stateAfter n))) fs)
      else do
        let before = stateAfter stop
            hdr = ehDecode stop
            v = vs VS.! stop
            err
              | v >= 13 && v <= 18 = envelopeError before hdr v
              | otherwise =
                  let TPraosState _ (TP.ChainDepState (Prtcl.PrtclState counters _ _) _ _) =
                        tpToState ops (headerStateChainDep before)
                      slotNo = blockSlot hdr
                      ovl = case Overlay.lookupInOverlaySchedule (epochFirst slotNo) (Map.keysSet dms) lvD f slotNo of
                        Nothing -> TPraosSlot
                        Just Overlay.NonActiveSlot -> TPraosNonActiveSlot
                        Just (Overlay.ActiveSlot gk) -> maybe TPraosNonActiveSlot TPraosActiveSlot (Map.lookup gk dms)
                  in HeaderProtocolError . tpProtocolErr ops $
                       tpraosChainTransitionError spkp maxEvo f lv (toNonce eta) counters ovl (tpView ops hdr)
                                                  (fs VS.! stop) (bs VS.! stop)
        pure (EpochValidationTPraos (EpochValidation vs bs stop (Left (stop, err, before))) fs)
  where
    fromSlot s = fromIntegral (fromEnum s) :: Word64
    fromBlock b = fromIntegral (fromEnum b) :: Word64
    epochFirst (SlotNo s) = SlotNo (if s < baseSlot then 0 else baseSlot + (s - baseSlot) `div` epochLen * epochLen)
    nonceBytes NeutralNonce = Nothing
    nonceBytes (Nonce h) = Just (hashToBytes h)
    decodeState cbor = case deserialiseOrFail (BSL.fromStrict cbor) of
      Right s -> s
      Left e  -> error ("PraosState CBOR returned by the batch fold: " ++ show e)
    -- validateEnvelope (HeaderValidation.hs:303-345) with TPraos's chainChecks errors
    envelopeError before hdr v =
      let oldTip = headerStateTip before
          p = Proxy @blk
          expB = case oldTip of
            Origin      -> expectedFirstBlockNo p
            NotOrigin t -> expectedNextBlockNo p (annTipInfo t) (getTipInfo hdr) (annTipBlockNo t)
          expS = case oldTip of
            Origin      -> minimumPossibleSlotNo p
            NotOrigin t -> minimumNextSlotNo p (annTipInfo t) (getTipInfo hdr) (annTipSlotNo t)
          TP.LedgerView {TP.lvChainChecks = TP.ChainChecksPParams {TP.ccMaxBHSize, TP.ccMaxBBSize,
                                                                   TP.ccProtocolVersion = ProtVer pvMajor _}} = lv
          (hsize, bsize) = tpSizes ops hdr
          other = tpEnvelopeErr ops <$>
            verdictToChainPredicateFailure (pvMajor, maxPV) (hsize, fromIntegral ccMaxBHSize)
                                           (bsize, fromIntegral ccMaxBBSize) v
      in maybe (error ("envelope verdict " ++ show v ++ " without its error")) HeaderEnvelopeError $
           verdictToHeaderEnvelopeError (expB, blockNo hdr) (expS, blockSlot hdr)
                                        (annTipHash <$> oldTip, headerPrevHash hdr) other v

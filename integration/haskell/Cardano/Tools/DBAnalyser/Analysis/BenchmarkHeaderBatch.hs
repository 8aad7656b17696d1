{-# LANGUAGE BangPatterns          #-}
{-# LANGUAGE DataKinds             #-}
{-# LANGUAGE FlexibleContexts      #-}
{-# LANGUAGE FlexibleInstances     #-}
{-# LANGUAGE LambdaCase            #-}
{-# LANGUAGE NamedFieldPuns        #-}
{-# LANGUAGE PatternSynonyms       #-}
{-# LANGUAGE RankNTypes            #-}
{-# LANGUAGE ScopedTypeVariables   #-}
{-# LANGUAGE TypeApplications      #-}
{-# LANGUAGE TypeFamilies          #-}
{-# LANGUAGE UndecidableInstances  #-}
{-# OPTIONS_GHC -Wno-orphans #-}

-- | db-analyser's header revalidation on the GPUs of one node: the analysis
-- @--benchmark-header-batch@ beside 'BenchmarkLedgerOps' (Analysis.hs:75-88, :479-607), wired in
-- by integration/haskell/db-analyser.patch (an 'AnalysisName' constructor, its 'runAnalysis'
-- equation, the Parsers.hs flag and the cabal stanza).
--
-- The analysis does what benchmarkLedgerOps does for every block -- keep the ledger state
-- (tick + reapply; no header validation on the CPU), forecast the ledger view a header is
-- validated under (Analysis.hs:564-572: @forecastFor (ledgerViewForecastAt lcfg (ledgerState
-- st)) slot@), validate the header (tickHeaderState + validateHeader) -- but it validates the
-- headers of a whole epoch in one GPU batch:
--
--   * The LedgerView of a Praos / TPraos epoch is the same for all of its headers: the
--     PoolDistr (@nesPd@) and the protocol parameters behind lvMaxHeaderSize / lvMaxBodySize /
--     lvProtocolVersion change only at an epoch boundary (the NEWEPOCH rule;
--     Shelley/Ledger/SupportsProtocol.hs:100-125).  The view forecast at the epoch's first slot,
--     from the ledger state before the epoch's first block, is the view of every header of the
--     epoch: one 'forecastFor' per epoch instead of one per header.
--   * The epoch's stored header bytes ('GetRawHeader') go into an arena that is reused epoch
--     after epoch and page-locked once per growth ('praosHostRegister'), so no pinning happens
--     inside a timed call (ehPin = 'PinnedByCaller'); 'validateEpochHeaders' /
--     'validateEpochHeadersTPraos' (Batch.Validate) run the epoch on the GPU(s) -- decode, OCert /
--     KES / VRF / leader crypto, then envelope + updateChainDepState -- and return the reference's
--     own 'HeaderState', or the first 'HeaderError'.
--   * Pipelining: epoch e validates on a worker thread while the stream reads, and the ledger
--     reapplies, the blocks of epoch e+1 (whose forecast needs the ledger state at its first
--     block).  Two arenas alternate: the worker reads one, the stream fills the other.
--   * Eras the batch does not cover (Byron's PBFT) and the first epoch of a new era, whose
--     chain-dependent state the hard-fork combinator translates at that epoch's first tick, run
--     the reference's own per-header path on the CPU, exactly as benchmarkLedgerOps does.
--
-- Output, one line per epoch:
--
--   epoch  path  headers  accepted  ms_forecast  ms_validate  headers/s
--
-- and the reference's 'HeaderError' for an invalid header; the analysis stops there, as
-- benchmarkLedgerOps does ("benchmark doesn't support invalid headers").
--
-- Shipped as source (no GHC where this repository is built).  Its foreign-call sequence per
-- epoch -- forecast -> praos_ticked_epoch_nonce -> praos_set_epoch (the epoch's PoolDistr) ->
-- praos_verify_header_bytes -> praos_validate_headers (the epoch's envelope limits), epoch e on a
-- worker while epoch e+1 streams, arenas registered once per growth -- is replayed from C by
-- integration/c/ffi_harness.c (phase "analysis", tests/test_gpu_views.py) on a chain whose
-- PoolDistr changes between epochs, and must equal praos_replay_immutable_views over the same
-- per-epoch views.
module Cardano.Tools.DBAnalyser.Analysis.BenchmarkHeaderBatch
  ( HeaderBatchArgs (..)
  , HasHeaderBatch (..)
  , EpochBatch
  , EpochOutcome (..)
  , benchmarkHeaderBatch
  ) where

import           Control.Concurrent (forkIO)
import           Control.Concurrent.MVar
import           Control.Exception (SomeException, throwIO, try)
import           Control.Monad (unless, when)
import           Control.Monad.Except (runExcept)
import qualified Data.ByteString as BS
import qualified Data.ByteString.Internal as BSI
import qualified Data.ByteString.Lazy as BSL
import qualified Data.ByteString.Short as SBS
import qualified Data.ByteString.Unsafe as BSU
import           Data.Fixed (Fixed (MkFixed))
import           Data.IORef
import qualified Data.Sequence as Seq
import           Data.SOP.Strict (NP (..), NS (..), (:.:) (..))
import qualified Data.Vector.Storable as VS
import qualified Data.Vector.Storable.Mutable as VSM
import           Data.Word (Word32, Word64, Word8)
import           Foreign.ForeignPtr.Unsafe (unsafeForeignPtrToPtr)
import           Foreign.Marshal.Utils (copyBytes)
import           Foreign.Ptr (Ptr, castPtr, plusPtr)
import           GHC.Clock (getMonotonicTimeNSec)
import qualified System.IO as IO
import           Text.Printf (hPrintf)

import           Cardano.Crypto.Hash (hashToBytes)
import           Cardano.Ledger.BaseTypes (activeSlotLog)
import           Cardano.Ledger.Shelley.API (computeStabilityWindow)
import qualified Cardano.Protocol.TPraos.API as TP
import           Cardano.Slotting.EpochInfo (epochInfoEpoch, epochInfoFirst, epochInfoSize)
import           Ouroboros.Consensus.Block
import           Ouroboros.Consensus.Byron.Ledger (ByronBlock)
import           Ouroboros.Consensus.Cardano.Block
import           Ouroboros.Consensus.Cardano.CanHardFork (CardanoHardForkConstraints)
import           Ouroboros.Consensus.Config
import           Ouroboros.Consensus.Config.SecurityParam (maxRollbacks)
import           Ouroboros.Consensus.Forecast (forecastFor)
import           Ouroboros.Consensus.HardFork.Abstract (HasHardForkHistory (..))
import           Ouroboros.Consensus.HardFork.Combinator
import           Ouroboros.Consensus.HardFork.Combinator.State (Current (..))
import qualified Ouroboros.Consensus.HardFork.Combinator.Util.Telescope as Telescope
import qualified Ouroboros.Consensus.HardFork.History as History
import           Ouroboros.Consensus.HeaderValidation
import           Ouroboros.Consensus.Ledger.Abstract
import           Ouroboros.Consensus.Ledger.Extended (ExtLedgerState (..))
import           Ouroboros.Consensus.Ledger.SupportsProtocol (LedgerSupportsProtocol (..))
import           Ouroboros.Consensus.Protocol.Praos (ConsensusConfig (..), Praos, PraosParams (..), PraosState,
                     Ticked (..))
import           Ouroboros.Consensus.Protocol.Praos.Common (MaxMajorProtVer (..))
import qualified Ouroboros.Consensus.Protocol.Praos.Views as Views
import           Ouroboros.Consensus.Protocol.TPraos (TPraos, TPraosParams (..), TPraosState)
import qualified Ouroboros.Consensus.Protocol.TPraos as TPraos
import           Ouroboros.Consensus.Shelley.Ledger (ShelleyBlock, ShelleyCompatible, ShelleyHash (..),
                     shelleyHeaderRaw)
import           Ouroboros.Consensus.Shelley.Protocol.Abstract (ProtocolHeaderSupportsEnvelope (..),
                     ProtocolHeaderSupportsProtocol (..))
import           Ouroboros.Consensus.TypeFamilyWrappers

import           Ouroboros.Consensus.Protocol.Praos.Batch
import           Ouroboros.Consensus.Protocol.Praos.Batch.Validate

-- | @--benchmark-header-batch [--out-file FILE] [--devices 0,1,...]@.
data HeaderBatchArgs = HeaderBatchArgs
  { hbOutFile :: Maybe FilePath
  , hbDevices :: [Int]          -- ^ one GPU, or a group (the 8 of a node: contiguous shards per epoch)
  } deriving Show

-- | What validating one epoch's headers returned: how many headers 'validateHeader' accepted,
-- the first invalid one's error (if any) and the 'HeaderState' after the accepted ones.
data EpochOutcome blk = EpochOutcome
  { eoAccepted :: !Int
  , eoError    :: !(Maybe (HeaderError blk))
  , eoState    :: !(HeaderState blk)
  }

-- | One epoch on the GPUs, from the 'HeaderState' before it.
type EpochBatch blk = PraosBatchCtx -> HeaderState blk -> EpochHeaders blk -> IO (EpochOutcome blk)

-- | Block types whose header validation the GPU batch takes over, one epoch at a time.
class HasHeaderBatch blk where
  -- | The batch of the epoch whose layout (first slot of the previous epoch, its number, the
  -- epoch length) and ticked ledger view are given, from the header state before the epoch;
  -- 'Nothing' when the epoch runs on the CPU (an era the batch does not cover, or the first
  -- epoch of an era whose chain-dependent state the hard-fork combinator has yet to translate).
  epochBatch :: TopLevelConfig blk -> (Word64, Word64, Word64) -> Ticked (LedgerView (BlockProtocol blk))
             -> HeaderState blk -> Maybe (EpochBatch blk)

-- ---------------------------------------------------------------- the analysis

-- | One epoch's headers as they stream in: the header bytes back to back in a Storable arena
-- page-locked once per growth, each header's offset and length, and the decoded headers (the
-- stopping header's error and the last accepted header's 'AnnTip' are built from them).
data EpochArena blk = EpochArena
  { eaBytes :: !(VSM.IOVector Word8)
  , eaPin   :: !(Maybe (Ptr Word8))        -- the registered buffer
  , eaOffs  :: !(VSM.IOVector Word64)
  , eaLens  :: !(VSM.IOVector Word32)
  , eaHdrs  :: !(Seq.Seq (Header blk))
  , eaLen   :: !Int
  , eaN     :: !Int
  }

newArena :: IO (EpochArena blk)
newArena = EpochArena <$> VSM.new (16 * 1024 * 1024) <*> pure Nothing <*> VSM.new 65536 <*> VSM.new 65536
                      <*> pure Seq.empty <*> pure 0 <*> pure 0

resetArena :: EpochArena blk -> EpochArena blk
resetArena a = a { eaHdrs = Seq.empty, eaLen = 0, eaN = 0 }

bufferPtr :: VSM.IOVector Word8 -> Ptr Word8
bufferPtr v = let (fp, _) = VSM.unsafeToForeignPtr0 v in unsafeForeignPtrToPtr fp

-- | Append one stored header (amortised doubling; a new byte buffer is registered, the old one
-- unregistered before it is dropped).
pushHeader :: PraosBatchCtx -> EpochArena blk -> Header blk -> BS.ByteString -> IO (EpochArena blk)
pushHeader ctx a hdr raw = do
  let l = BS.length raw
      grow v need = if VSM.length v >= need then pure v else VSM.grow v (max need (VSM.length v))
  bytes <- grow (eaBytes a) (eaLen a + l)
  pin <- if eaPin a == Just (bufferPtr bytes) then pure (eaPin a) else do
    mapM_ (praosHostUnregister ctx) (eaPin a)
    praosHostRegister ctx (bufferPtr bytes) (VSM.length bytes)
    pure (Just (bufferPtr bytes))
  offs <- grow (eaOffs a) (eaN a + 1)
  lens <- grow (eaLens a) (eaN a + 1)
  VSM.unsafeWith bytes $ \dst -> BSU.unsafeUseAsCString raw $ \src ->
    copyBytes (dst `plusPtr` eaLen a) (castPtr src) l
  VSM.unsafeWrite offs (eaN a) (fromIntegral (eaLen a))
  VSM.unsafeWrite lens (eaN a) (fromIntegral l)
  pure a { eaBytes = bytes, eaPin = pin, eaOffs = offs, eaLens = lens, eaHdrs = eaHdrs a Seq.|> hdr
         , eaLen = eaLen a + l, eaN = eaN a + 1 }

-- | The epoch's headers as 'EpochHeaders' over the arena's own (registered) buffer.
epochHeaders :: EpochArena blk -> IO (EpochHeaders blk)
epochHeaders a = do
  let n = eaN a
  offs <- VS.freeze (VSM.slice 0 n (eaOffs a))
  lens <- VS.freeze (VSM.slice 0 n (eaLens a))
  let (fp, _) = VSM.unsafeToForeignPtr0 (eaBytes a)
  pure EpochHeaders { ehArena = BSI.fromForeignPtr fp 0 (eaLen a), ehOffset = offs, ehLength = lens
                    , ehDecode = Seq.index (eaHdrs a), ehPin = PinnedByCaller }

-- | The epoch in progress: on the GPUs (its batch and forecast time) or on the CPU (headers
-- seen, accepted, milliseconds of validation).
data EpochMode blk
  = OnGpu !Word64 (EpochBatch blk) !Double
  | OnCpu !Word64 !Int !Int !Double

-- | The analysis.  @stream@ is Analysis.hs's @processAll db registry ((,) <$> GetBlock <*>
-- GetRawHeader) initLedger limit@ (:753-766; the ImmutableDB stream :815-847).
benchmarkHeaderBatch
  :: forall blk.
     ( HasHeaderBatch blk, LedgerSupportsProtocol blk, HasAnnTip blk, GetPrevHash blk
     , HasHardForkHistory blk, Show (HeaderError blk) )
  => HeaderBatchArgs
  -> TopLevelConfig blk
  -> ExtLedgerState blk
  -> (forall st. st -> (st -> (blk, BSL.ByteString) -> IO st) -> IO st)
  -> IO ()
benchmarkHeaderBatch HeaderBatchArgs {hbOutFile, hbDevices} cfg initLedger stream =
  withOut hbOutFile $ \h -> withPraosBatchDevices hbDevices $ \ctx -> do
    IO.hPutStrLn h ("# devices " ++ show hbDevices ++ " (" ++ show (praosBatchMembers ctx) ++ " contexts)")
    IO.hPutStrLn h "epoch\tpath\theaders\taccepted\tms_forecast\tms_validate\theaders/s"
    fillRef <- newArena >>= newIORef                  -- the arena the stream fills
    spareRef <- newArena >>= newIORef                 -- the one the worker reads (or read last)
    ledgerRef <- newIORef (ledgerState initLedger)
    hstRef <- newIORef (headerState initLedger)       -- after the last finished epoch
    modeRef <- newIORef Nothing                       -- the epoch in progress
    inflight <- newIORef Nothing                      -- the epoch on the worker
    stopped <- newIORef False
    let lcfg = topLevelConfigLedger cfg
        ccfg = topLevelConfigProtocol cfg
        -- the ledger view at a slot, forecast from a ledger state (Analysis.hs:564-572)
        forecast st slot = case runExcept (forecastFor (ledgerViewForecastAt lcfg st) slot) of
          Left err -> throwIO (userError ("header batch: " ++ show slot ++ " beyond the forecast range: " ++ show err))
          Right tlv -> pure tlv
        -- the slot's epoch and the layout the batch fold counts epochs in: fixed-length epochs
        -- from the previous epoch's first slot (the header state's last slot, always before the
        -- epoch, then ticks exactly once)
        layout st slot = either throwIO pure $ do
          let ei = History.summaryToEpochInfo (hardForkSummary lcfg st)
          EpochNo e <- runExcept (epochInfoEpoch ei slot)
          let prev = if e == 0 then 0 else e - 1
          SlotNo first <- runExcept (epochInfoFirst ei (EpochNo prev))
          EpochSize size <- runExcept (epochInfoSize ei (EpochNo e))
          pure (e, (first, prev, size))
        report e path n EpochOutcome {eoAccepted, eoError, eoState} tFc ms = do
          hPrintf h "%d\t%s\t%d\t%d\t%.3f\t%.3f\t%.0f\n" e (path :: String) n eoAccepted (tFc :: Double) (ms :: Double)
                  (fromIntegral n / max 1e-9 (ms / 1e3) :: Double)
          writeIORef hstRef eoState
          case eoError of
            Nothing -> pure ()
            Just err -> do
              hPrintf h "# epoch %d: header %d is invalid: %s\n" e eoAccepted (show err)
              writeIORef stopped True
        -- waits for the epoch on the worker and reports it
        joinWorker = readIORef inflight >>= \case
          Nothing -> pure ()
          Just (e, n, tFc, mv) -> do
            writeIORef inflight Nothing
            (o, ms) <- takeMVar mv >>= either throwIO pure
            report e "gpu" n o tFc ms
        -- the epoch in progress is complete: a GPU epoch goes to the worker (after the previous
        -- one, whose state it starts from), a CPU epoch is reported
        finishEpoch = readIORef modeRef >>= \case
          Just (OnGpu e batch tFc) -> do
            joinWorker
            done <- readIORef stopped
            a <- readIORef fillRef
            unless (done || eaN a == 0) $ do
              hst <- readIORef hstRef
              hs <- epochHeaders a
              mv <- newEmptyMVar
              _ <- forkIO $ do
                r <- try $ do
                  t0 <- getMonotonicTimeNSec
                  !o <- batch ctx hst hs
                  t1 <- getMonotonicTimeNSec
                  pure (o, fromIntegral (t1 - t0) / 1e6 :: Double)
                putMVar mv (r :: Either SomeException (EpochOutcome blk, Double))
              writeIORef inflight (Just (e, eaN a, tFc, mv))
              -- the stream fills the other arena (free: its worker has been joined above)
              spare <- readIORef spareRef
              writeIORef spareRef a
              writeIORef fillRef (resetArena spare)
          Just (OnCpu e n ok ms) | n > 0 -> do
            done <- readIORef stopped
            unless done $ do
              hst <- readIORef hstRef
              report e "cpu" n (EpochOutcome ok Nothing hst) 0 ms
          _ -> pure ()
        onBlock () (blk, raw) = readIORef stopped >>= \done -> unless done $ do
          st <- readIORef ledgerRef
          let slot = blockSlot blk
              hdr = getHeader blk
          (e, ei) <- layout st slot
          mode <- readIORef modeRef
          let epochOf = \case
                OnGpu x _ _ -> x
                OnCpu x _ _ _ -> x
          when (fmap epochOf mode /= Just e) $ do
            finishEpoch                               -- the previous epoch goes to the worker
            t0 <- getMonotonicTimeNSec
            tlv <- forecast st slot
            t1 <- getMonotonicTimeNSec
            -- the last joined header state: while the worker still has the previous epoch it is
            -- the state before that one, in the same era (a batch never changes the era), which
            -- is all epochBatch reads of it; the batch itself gets the state after the previous
            -- epoch when it is launched
            hst <- readIORef hstRef
            writeIORef modeRef . Just $ case epochBatch cfg ei tlv hst of
              Just batch -> OnGpu e batch (fromIntegral (t1 - t0) / 1e6)
              Nothing    -> OnCpu e 0 0 0
          done' <- readIORef stopped
          unless done' $ readIORef modeRef >>= \case
            Just (OnGpu {}) -> readIORef fillRef >>= \a -> pushHeader ctx a hdr (BSL.toStrict raw) >>= writeIORef fillRef
            Just (OnCpu x n ok ms) -> do
              -- the reference's per-header path: the view at this header's slot, tick, validateHeader
              joinWorker
              tlv <- forecast st slot
              hst <- readIORef hstRef
              t0 <- getMonotonicTimeNSec
              let r = runExcept (validateHeader cfg tlv hdr (tickHeaderState ccfg tlv slot hst))
              t1 <- either (const getMonotonicTimeNSec) (\s -> s `seq` getMonotonicTimeNSec) r
              let ms' = ms + fromIntegral (t1 - t0) / 1e6
              case r of
                Right hst' -> writeIORef hstRef hst' >> writeIORef modeRef (Just (OnCpu x (n + 1) (ok + 1) ms'))
                Left err -> do
                  report x "cpu" (n + 1) (EpochOutcome ok (Just err) hst) 0 ms'
                  writeIORef modeRef Nothing
            Nothing -> pure ()
          -- the ledger state after the block (tick + reapply: a stored block was valid)
          writeIORef ledgerRef $! tickThenReapply lcfg blk st
    stream () onBlock
    finishEpoch
    joinWorker
    done <- readIORef stopped
    when done $ IO.hPutStrLn h "# stopped at the first invalid header"
    mapM_ (\r -> readIORef r >>= mapM_ (praosHostUnregister ctx) . eaPin) [fillRef, spareRef]
  where
    withOut (Just f) k = IO.withFile f IO.WriteMode k
    withOut Nothing k = k IO.stdout

-- ---------------------------------------------------------------- per-era batches

-- | A Praos epoch: 'validateEpochHeaders' under the forecast 'Views.LedgerView' (the block
-- ops may depend on the header state before the epoch: the hard-fork combinator's telescope).
praosEpochBatch :: forall blk c. ( BasicEnvelopeValidation blk, HasAnnTip blk, GetPrevHash blk, HasHeader (Header blk)
                                 , TP.PraosCrypto c )
                => PraosParams -> (Word64, Word64, Word64) -> Views.LedgerView c
                -> (HeaderState blk -> PraosBlockOps blk c) -> EpochBatch blk
praosEpochBatch pp (first, prev, size) lv opsFor ctx st0 hs = do
  let window = computeStabilityWindow (maxRollbacks (praosSecurityParam pp)) (praosLeaderF pp)
  ev <- validateEpochHeaders ctx (opsFor st0) pp (praosLeaderF pp) (first, prev, size, window)
                             (getMaxMajorProtVer (praosMaxMajorPV pp)) lv st0 hs
  pure $ case evOutcome ev of
    Right st          -> EpochOutcome (evAccepted ev) Nothing st
    Left (k, err, st) -> EpochOutcome k (Just err) st

-- | A TPraos epoch: 'validateEpochHeadersTPraos' under the forecast 'TP.LedgerView'.
tpraosEpochBatch :: forall blk c. ( BasicEnvelopeValidation blk, HasAnnTip blk, GetPrevHash blk, HasHeader (Header blk)
                                  , TP.PraosCrypto c )
                 => TPraosParams -> (Word64, Word64, Word64) -> TP.LedgerView c
                 -> (HeaderState blk -> TPraosBlockOps blk c) -> EpochBatch blk
tpraosEpochBatch TPraosParams {tpraosSlotsPerKESPeriod, tpraosMaxKESEvo, tpraosLeaderF, tpraosSecurityParam,
                               tpraosMaxMajorPV}
                 (first, prev, size) lv opsFor ctx st0 hs = do
  let MkFixed cRaw = activeSlotLog tpraosLeaderF
      window = computeStabilityWindow (maxRollbacks tpraosSecurityParam) tpraosLeaderF
  evt <- validateEpochHeadersTPraos ctx (opsFor st0) (tpraosSlotsPerKESPeriod, tpraosMaxKESEvo, tpraosLeaderF) cRaw
                                    (first, prev, size, window) (getMaxMajorProtVer tpraosMaxMajorPV) lv st0 hs
  let ev = evtValidation evt
  pure $ case evOutcome ev of
    Right st          -> EpochOutcome (evAccepted ev) Nothing st
    Left (k, err, st) -> EpochOutcome k (Just err) st

-- | 'PraosBlockOps' of a single-era Praos block: every conversion is the identity.
shelleyPraosOps :: ShelleyCompatible (Praos c) era => PraosBlockOps (ShelleyBlock (Praos c) era) c
shelleyPraosOps = PraosBlockOps
  { pbView = protocolHeaderView @(Praos _) . shelleyHeaderRaw
  , pbHashBytes = hashToBytes . unShelleyHash
  , pbSizes = \hdr -> let r = shelleyHeaderRaw hdr in (pHeaderSize r, pHeaderBlockSize r)
  , pbToState = id
  , pbFromState = id
  , pbProtocolErr = id
  , pbEnvelopeErr = id
  }

-- | 'TPraosBlockOps' of a single-era TPraos block.
shelleyTPraosOps :: ShelleyCompatible (TPraos c) era => TPraosBlockOps (ShelleyBlock (TPraos c) era) c
shelleyTPraosOps = TPraosBlockOps
  { tpView = shelleyHeaderRaw
  , tpHashBytes = hashToBytes . unShelleyHash
  , tpSizes = \hdr -> let r = shelleyHeaderRaw hdr in (pHeaderSize r, pHeaderBlockSize r)
  , tpToState = id
  , tpFromState = id
  , tpProtocolErr = id
  , tpEnvelopeErr = id
  }

-- | The Cardano block's ops for a Praos era (Babbage, Conway): the era's header out of the
-- hard-fork header, the era's state out of the telescope's current era and back in (the past
-- eras and the era's start kept: an epoch never crosses an era boundary), errors injected at the
-- era's index.
cardanoPraosOps
  :: forall c era. (CardanoHardForkConstraints c, ShelleyCompatible (Praos c) era)
  => (forall f. f (ShelleyBlock (Praos c) era) -> NS f (CardanoEras c))
  -> (Header (CardanoBlock c) -> Header (ShelleyBlock (Praos c) era))
  -> (HardForkChainDepState (CardanoEras c) -> PraosState c)
  -> (HardForkChainDepState (CardanoEras c) -> PraosState c -> HardForkChainDepState (CardanoEras c))
  -> HeaderState (CardanoBlock c) -> PraosBlockOps (CardanoBlock c) c
cardanoPraosOps tag projH projS injS st0 = PraosBlockOps
  { pbView = protocolHeaderView @(Praos c) . shelleyHeaderRaw . projH
  , pbHashBytes = SBS.fromShort . getOneEraHash
  , pbSizes = \hdr -> let r = shelleyHeaderRaw (projH hdr) in (pHeaderSize r, pHeaderBlockSize r)
  , pbToState = projS
  , pbFromState = injS (headerStateChainDep st0)
  , pbProtocolErr = HardForkValidationErrFromEra . OneEraValidationErr . tag . WrapValidationErr
  , pbEnvelopeErr = HardForkEnvelopeErrFromEra . OneEraEnvelopeErr . tag . WrapEnvelopeErr
  }

-- | The Cardano block's ops for a TPraos era (Shelley..Alonzo).
cardanoTPraosOps
  :: forall c era. (CardanoHardForkConstraints c, ShelleyCompatible (TPraos c) era)
  => (forall f. f (ShelleyBlock (TPraos c) era) -> NS f (CardanoEras c))
  -> (Header (CardanoBlock c) -> Header (ShelleyBlock (TPraos c) era))
  -> (HardForkChainDepState (CardanoEras c) -> TPraosState c)
  -> (HardForkChainDepState (CardanoEras c) -> TPraosState c -> HardForkChainDepState (CardanoEras c))
  -> HeaderState (CardanoBlock c) -> TPraosBlockOps (CardanoBlock c) c
cardanoTPraosOps tag projH projS injS st0 = TPraosBlockOps
  { tpView = shelleyHeaderRaw . projH
  , tpHashBytes = SBS.fromShort . getOneEraHash
  , tpSizes = \hdr -> let r = shelleyHeaderRaw (projH hdr) in (pHeaderSize r, pHeaderBlockSize r)
  , tpToState = projS
  , tpFromState = injS (headerStateChainDep st0)
  , tpProtocolErr = HardForkValidationErrFromEra . OneEraValidationErr . tag . WrapValidationErr
  , tpEnvelopeErr = HardForkEnvelopeErrFromEra . OneEraEnvelopeErr . tag . WrapEnvelopeErr
  }

-- ---------------------------------------------------------------- instances

-- | Praos eras (Babbage, Conway) as a single-era block.
instance (ShelleyCompatible (Praos c) era, TP.PraosCrypto c) => HasHeaderBatch (ShelleyBlock (Praos c) era) where
  epochBatch cfg ei (TickedPraosLedgerView lv) _ =
    Just $ praosEpochBatch (praosParams (configConsensus cfg)) ei lv (const shelleyPraosOps)

-- | TPraos eras (Shelley..Alonzo) as a single-era block (db-analyser's @shelley@ block type).
instance (ShelleyCompatible (TPraos c) era, TP.PraosCrypto c) => HasHeaderBatch (ShelleyBlock (TPraos c) era) where
  epochBatch cfg ei (TPraos.TickedPraosLedgerView lv) _ =
    Just $ tpraosEpochBatch (TPraos.tpraosParams (configConsensus cfg)) ei lv (const shelleyTPraosOps)

-- | Byron (PBFT): the CPU path.
instance HasHeaderBatch ByronBlock where
  epochBatch _ _ _ _ = Nothing

-- | The Cardano block: the era of the epoch's ledger view decides, and the header state's
-- current era must be the same one (else the combinator has yet to translate the state: the
-- first epoch after a hard fork runs on the CPU).
instance CardanoHardForkConstraints c => HasHeaderBatch (CardanoBlock c) where
  epochBatch cfg ei tlv hst = case (viewTip, stateTip) of
    (TagBabbage (Current _ (Comp (WrapTickedLedgerView (TickedPraosLedgerView lv)))), TagBabbage _) ->
      Just $ praosEpochBatch (partial babbageP) ei lv $
        cardanoPraosOps TagBabbage (\(HeaderBabbage x) -> x)
          (\s -> case getHardForkState s of
             TeleBabbage _ _ _ _ _ (Current _ (WrapChainDepState x)) -> x
             _ -> error "header batch: not a Babbage state")
          (\s x -> HardForkState $ case getHardForkState s of
             TeleBabbage a b c' d e' (Current t _) -> TeleBabbage a b c' d e' (Current t (WrapChainDepState x))
             _ -> error "header batch: not a Babbage state")
    (TagConway (Current _ (Comp (WrapTickedLedgerView (TickedPraosLedgerView lv)))), TagConway _) ->
      Just $ praosEpochBatch (partial conwayP) ei lv $
        cardanoPraosOps TagConway (\(HeaderConway x) -> x)
          (\s -> case getHardForkState s of
             TeleConway _ _ _ _ _ _ (Current _ (WrapChainDepState x)) -> x
             _ -> error "header batch: not a Conway state")
          (\s x -> HardForkState $ case getHardForkState s of
             TeleConway a b c' d e' f' (Current t _) -> TeleConway a b c' d e' f' (Current t (WrapChainDepState x))
             _ -> error "header batch: not a Conway state")
    (TagShelley (Current _ (Comp (WrapTickedLedgerView (TPraos.TickedPraosLedgerView lv)))), TagShelley _) ->
      Just $ tpraosEpochBatch (partial shelleyP) ei lv $
        cardanoTPraosOps TagShelley (\(HeaderShelley x) -> x)
          (\s -> case getHardForkState s of
             TeleShelley _ (Current _ (WrapChainDepState x)) -> x
             _ -> error "header batch: not a Shelley state")
          (\s x -> HardForkState $ case getHardForkState s of
             TeleShelley a (Current t _) -> TeleShelley a (Current t (WrapChainDepState x))
             _ -> error "header batch: not a Shelley state")
    (TagAllegra (Current _ (Comp (WrapTickedLedgerView (TPraos.TickedPraosLedgerView lv)))), TagAllegra _) ->
      Just $ tpraosEpochBatch (partial allegraP) ei lv $
        cardanoTPraosOps TagAllegra (\(HeaderAllegra x) -> x)
          (\s -> case getHardForkState s of
             TeleAllegra _ _ (Current _ (WrapChainDepState x)) -> x
             _ -> error "header batch: not an Allegra state")
          (\s x -> HardForkState $ case getHardForkState s of
             TeleAllegra a b (Current t _) -> TeleAllegra a b (Current t (WrapChainDepState x))
             _ -> error "header batch: not an Allegra state")
    (TagMary (Current _ (Comp (WrapTickedLedgerView (TPraos.TickedPraosLedgerView lv)))), TagMary _) ->
      Just $ tpraosEpochBatch (partial maryP) ei lv $
        cardanoTPraosOps TagMary (\(HeaderMary x) -> x)
          (\s -> case getHardForkState s of
             TeleMary _ _ _ (Current _ (WrapChainDepState x)) -> x
             _ -> error "header batch: not a Mary state")
          (\s x -> HardForkState $ case getHardForkState s of
             TeleMary a b c' (Current t _) -> TeleMary a b c' (Current t (WrapChainDepState x))
             _ -> error "header batch: not a Mary state")
    (TagAlonzo (Current _ (Comp (WrapTickedLedgerView (TPraos.TickedPraosLedgerView lv)))), TagAlonzo _) ->
      Just $ tpraosEpochBatch (partial alonzoP) ei lv $
        cardanoTPraosOps TagAlonzo (\(HeaderAlonzo x) -> x)
          (\s -> case getHardForkState s of
             TeleAlonzo _ _ _ _ (Current _ (WrapChainDepState x)) -> x
             _ -> error "header batch: not an Alonzo state")
          (\s x -> HardForkState $ case getHardForkState s of
             TeleAlonzo a b c' d (Current t _) -> TeleAlonzo a b c' d (Current t (WrapChainDepState x))
             _ -> error "header batch: not an Alonzo state")
    _ -> Nothing                                      -- Byron, or an era boundary: the CPU path
    where
      viewTip = Telescope.tip (getHardForkState (tickedHardForkLedgerViewPerEra tlv))
      stateTip = Telescope.tip (getHardForkState (headerStateChainDep hst))
      PerEraConsensusConfig (_byronP :* shelleyP :* allegraP :* maryP :* alonzoP :* babbageP :* conwayP :* Nil) =
        hardForkConsensusConfigPerEra (configConsensus cfg)
      partial :: WrapPartialConsensusConfig x -> PartialConsensusConfig (BlockProtocol x)
      partial (WrapPartialConsensusConfig p) = p
